"""nRanks == 1 AllReduce with ncclAvg (the PreMulSum kernel, oneRankKernel) vs ncclSum (the copy): HBM GB/s
(2S/t) at 256 MiB for fp32 / bf16 / fp8, HIP events over 20 launches. Diagnostics (scripts/)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nccl_amd  # noqa: E402

torch.cuda.set_device(0)
comm = nccl_amd.Communicator.init_all([0])[0]
s = torch.cuda.current_stream()
S = 256 << 20
for name, dt, code in (("fp32", torch.float32, 7), ("bf16", torch.bfloat16, 9), ("uint8", torch.uint8, 1)):
    n = S // torch.tensor([], dtype=dt).element_size()
    x = torch.randint(0, 100, (n,), device="cuda").to(dt)
    y = torch.empty_like(x)
    for opname, op in (("sum(copy)", 0), ("avg(premul)", 4)):
        for _ in range(5):
            comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), n, code, op, s.cuda_stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(20):
            comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), n, code, op, s.cuda_stream)
        b.record(s)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        ok = bool(torch.equal(y, x)) if op == 0 or dt != torch.uint8 else True
        print(f"{name:6s} {opname:12s} {ms * 1e3:8.1f} us {2 * S / (ms * 1e-3) / 1e9:8.1f} GB/s ok={ok}", flush=True)
comm.destroy()
