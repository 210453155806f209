"""Re-run one parity case (or a short sequence) on a fresh single-process communicator.
Usage: python scripts/repro_case.py NRANKS 'ENV_JSON' 'CASES_JSON'   CASES: [[coll, dtype, op, count, mis, root], ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "10000")
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
n = int(sys.argv[1])
os.environ.update(json.loads(sys.argv[2]))
import torch  # noqa: E402

import nccl_amd  # noqa: E402
from tests import gpu_cases as G  # noqa: E402

torch.cuda.set_device(0)
comms = nccl_amd.Communicator.init_all([0] * n)
cs = list(zip(comms, [torch.cuda.Stream() for _ in range(n)]))
bad = 0
for i, (coll, dt, op, count, mis, root) in enumerate(json.loads(sys.argv[3])):
    errs = G.run_case(cs, coll, dt, op, count, mis, seed=77 + i, root=root)
    print(f"{coll} dt={dt} op={op} count={count} mis={mis} root={root}: {'OK' if not errs else errs[:2]}", flush=True)
    bad += bool(errs)
for c in comms:
    c.destroy()
sys.exit(1 if bad else 0)
