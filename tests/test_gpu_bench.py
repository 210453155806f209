"""bench.py's N>1 harness end to end on the one-GPU box: torchrun with 2 ranks (each a process on the same
GPU), quick suite. Guards the unique-id exchange, barriers, max-over-ranks timing, the suite's extra
communicators and windows, and the one JSON line the driver parses — the code the round-end multi-GPU
run executes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_quick(built):
    env = dict(os.environ, NCCL_AMD_SPIN_TIMEOUT_MS="20000")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--quick-suite", "--no-cpu-baseline"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["check"] == "pass" and d["value"] > 0 and d["unit"] == "GB/s"
    assert d["roofline"]["bound"] == "hbm" and "xgmi" in d["roofline"]
    s = d["suite"]
    assert "error" not in s, s
    assert s["rs_ag_bf16"]["check"] == "pass" and s["reduce_int32"]["check"].startswith("pass")
    assert s["symmetric_window"]["check"].startswith("pass")
    assert s["group_aggregation"]["aggregated_us_per_group"] > 0
