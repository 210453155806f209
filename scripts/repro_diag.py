"""Diagnose one failing AllReduce: print, for the first mismatches, every rank's input, the expected and the
received value, and which simple combination the received value matches.
Usage: python scripts/repro_diag.py NRANKS 'ENV_JSON' DTYPE COUNT"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "10000")
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
n = int(sys.argv[1])
os.environ.update(json.loads(sys.argv[2]))
dt, count = int(sys.argv[3]), int(sys.argv[4])
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nccl_amd  # noqa: E402
import oracle  # noqa: E402
from tests import gpu_cases as G  # noqa: E402

torch.cuda.set_device(0)
comms = nccl_amd.Communicator.init_all([0] * n)
streams = [torch.cuda.Stream() for _ in range(n)]
ins = G.make_inputs(n, dt, count, 5)
want = oracle.all_reduce(ins, dt, 0)
npdt = oracle.NP_STORAGE[dt]
bufs = [G.to_device(x, torch.device("cuda", 0)) for x in ins]
outs = [G.to_device(np.zeros(count, dtype=npdt), torch.device("cuda", 0)) for _ in range(n)]
torch.cuda.synchronize()
with nccl_amd.group():
    for c, s, (_, sv), (_, rv) in zip(comms, streams, bufs, outs):
        c.all_reduce_raw(sv.data_ptr(), rv.data_ptr(), count, dt, 0, s.cuda_stream)
torch.cuda.synchronize()
got = G.from_device(outs[0][1], npdt)
bad = np.nonzero(got != want)[0]
print(f"{bad.size} mismatches of {count}")
for i in bad[:12]:
    vals = [int(x[i]) for x in ins]
    print(f"i={i} (pack {i * np.dtype(npdt).itemsize // 16}, byte {i * np.dtype(npdt).itemsize}) ins={vals} want={int(want[i])} "
          f"got={int(got[i])} got==in0:{int(got[i]) == vals[0]} got==in1:{int(got[i]) == vals[1] if n > 1 else None}")
# runs of bad indices
if bad.size:
    runs, start = [], bad[0]
    for a, b in zip(bad[:-1], bad[1:]):
        if b != a + 1:
            runs.append((int(start), int(a)))
            start = b
    runs.append((int(start), int(bad[-1])))
    print("first runs:", runs[:20], "n runs", len(runs))
for c in comms:
    c.destroy()
