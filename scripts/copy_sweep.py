"""Sweep of the nRanks==1 copy kernel variants (NCCL_AMD_COPY_VARIANT / NCCL_AMD_COPY_GRID) at 64 and
256 MiB, timed with HIP events on the launch stream, next to hipMemcpyAsync D2D (torch copy_)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import nccl_amd

torch.cuda.set_device(0)
comm = nccl_amd.Communicator.init_all([0])[0]
st = torch.cuda.current_stream()
res = []
for mib in (64, 256):
    n = mib * 2**20 // 4
    a = torch.empty(n, device="cuda").uniform_(-1, 1)
    b = torch.empty_like(a)
    def t(fn, it=40):
        for _ in range(5): fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(it): fn()
        e1.record(st); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / it
        return round(2 * mib * 2**20 / (ms * 1e-3) / 1e9, 1)
    res.append({"mib": mib, "variant": "hipMemcpyAsync", "GBps": t(lambda: b.copy_(a))})
    for var in (0, 1, 2, 3):
        for grid in (512, 1024, 2048, 4096, 8192):
            os.environ["NCCL_AMD_COPY_VARIANT"] = str(var)
            os.environ["NCCL_AMD_COPY_GRID"] = str(grid)
            gb = t(lambda: comm.all_reduce_raw(a.data_ptr(), b.data_ptr(), n, 7, 0, st.cuda_stream))
            res.append({"mib": mib, "variant": var, "grid": grid, "GBps": gb})
            assert torch.equal(a, b)
    del a, b
for r in res:
    print(json.dumps(r))
