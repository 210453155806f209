"""Build-time resource check of the channel kernels (no GPU): every collKernel / llKernel / symKernel
instantiation must fit two 512-thread workgroups per CU (>= 4 waves per SIMD, <= 128 VGPRs) without
spilling VGPRs to scratch. Several ranks on one GPU rely on it: the host plans up to CUs / ranksPerGPU channels
per launch and every channel of every rank must be resident at once, or the ranks wait on each other
forever (a 1-byte kernel at 256 VGPRs did exactly that before the kCoResident budget). The report comes
from the compiler (-Rpass-analysis=kernel-resource-usage, written to build/<name>.usage by `make`)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHANNEL_KERNELS = ("collKernel", "llKernel", "symKernel")


def _reports():
    out = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "build", "*.usage"))):
        cur = None
        for line in open(path, errors="replace"):
            m = re.search(r"remark: Function Name: (\S+)", line)
            if m:
                cur = out.setdefault(m.group(1), {"file": os.path.basename(path)})
                continue
            m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[-Rpass", line)
            if m and cur is not None:
                cur[m.group(1).strip()] = m.group(2)
    return out


def test_channel_kernels_fit_two_workgroups_per_cu():
    reps = _reports()
    if not reps:
        pytest.skip("no build/*.usage reports: run `make` first")
    chan = {k: v for k, v in reps.items() if any(n in k for n in CHANNEL_KERNELS)}
    assert len(chan) >= 100, f"only {len(chan)} channel kernels in the reports"
    bad = []
    for name, r in chan.items():
        occ = int(r.get("Occupancy", 0))
        vgpr = int(r.get("VGPRs", 999))
        spill = int(r.get("VGPRs Spill", 0))      # SGPR spills land in VGPR lanes, not memory
        scratch = int(r.get("ScratchSize", 0))
        if occ < 4 or vgpr > 128 or spill or scratch:
            bad.append(f"{r['file']}: {name}: VGPRs {vgpr} occupancy {occ} VGPR spills {spill} scratch {scratch}")
    assert not bad, "\n".join(bad[:20])
