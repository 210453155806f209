"""Probe: single-process 2-rank AllReduce at growing sizes (multi-step channel pipelines), reporting the
async error and correctness per size. Usage: python scripts/big_probe.py [dtype_code] [sizes_MiB...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "5000")
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
import torch  # noqa: E402

import nccl_amd  # noqa: E402

dt = int(sys.argv[1]) if len(sys.argv) > 1 else 7
sizes = [int(x) for x in sys.argv[2:]] or [256, 512, 1024, 2048, 2100]
tdt = {7: torch.float32, 1: torch.uint8, 2: torch.int32}[dt]
es = torch.tensor([], dtype=tdt).element_size()
torch.cuda.set_device(0)
comms = nccl_amd.Communicator.init_all([0, 0])
streams = [torch.cuda.Stream() for _ in range(2)]
for mib in sizes:
    count = mib * (1 << 20) // es + 4099
    xs = [torch.full((count,), r + 1, dtype=tdt, device="cuda") for r in range(2)]
    ys = [torch.empty_like(x) for x in xs]
    torch.cuda.synchronize()
    t0 = time.time()
    with nccl_amd.group():
        for c, s, x, y in zip(comms, streams, xs, ys):
            c.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, dt, 0, s.cuda_stream)
    torch.cuda.synchronize()
    errs = [c.async_error() for c in comms]
    ok = all(bool((y == 3).all()) for y in ys) if not any(errs) else False
    bad = [int((y != 3).sum()) for y in ys]
    print(f"{mib} MiB count {count}: async {errs} ok {ok} wrong {bad} {time.time() - t0:.2f}s", flush=True)
    if any(errs):
        break
    del xs, ys
for c in comms:
    c.destroy()
