"""Two ranks of one process on the box's one GPU (ncclCommInitAll([0, 0])): the n=2 AllReduce kernels
(staged direct, symmetric windows, ncclCommRegister'd buffers, LL) on the metric's 256 MiB fp32 per rank, for rocprofv3 traces.
Every "remote" byte is local HBM here, so this profiles the protocol and the kernels' HBM traffic, not
xGMI. No process is spawned (safe under rocprofv3)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"

import torch  # noqa: E402

import nccl_amd  # noqa: E402

MIB = 1 << 20


def main():
    steps = int(os.environ.get("STEPS", "20"))
    mode = os.environ.get("MODE", "direct")  # direct | sym | reg | ll
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0])
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    S = (64 * 1024 if mode == "ll" else 256 * MIB)
    c = S // 4
    bufs = [torch.empty(2 * S, dtype=torch.uint8, device="cuda") for _ in comms]
    if mode == "sym":
        with nccl_amd.group():
            wins = [cm.register_window(b.data_ptr(), 2 * S) for cm, b in zip(comms, bufs)]
    if mode == "reg":  # ncclCommRegister only: the zero-copy kernel in registered mode (pointer exchange)
        regs = [cm.register_buffer(b.data_ptr(), 2 * S) for cm, b in zip(comms, bufs)]
    for r, b in enumerate(bufs):
        b[:S].view(torch.float32).fill_(r + 1)
    torch.cuda.synchronize()

    def step():
        with nccl_amd.group():
            for cm, s, b in zip(comms, streams, bufs):
                cm.all_reduce_raw(b.data_ptr(), b.data_ptr() + S, c, 7, 0, s.cuda_stream)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in streams]
    for (a, _), s in zip(ev, streams):
        a.record(s)
    for _ in range(steps):
        step()
    for (_, b), s in zip(ev, streams):
        b.record(s)
    torch.cuda.synchronize()
    ms = max(a.elapsed_time(b) for a, b in ev) / steps
    ok = all(bool((b[S:].view(torch.float32) == 3.0).all()) for b in bufs)
    print(json.dumps({"mode": mode, "bytes_per_rank": S, "ms": round(ms, 4),
                      "busbw_GBps": round(S / (ms * 1e-3) / 1e9, 2), "check": ok}), flush=True)
    if mode == "sym":
        for cm, w in zip(comms, wins):
            cm.deregister_window(w)
    if mode == "reg":
        for cm, h in zip(comms, regs):
            cm.deregister_buffer(h)
    for cm in comms:
        cm.destroy()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
