"""One rank of an n-process AllReduce on the one-GPU box (n = $NRANKS, default 2), rendezvous through a file (no
launcher, so one of the processes can run under rocprofv3 without any process being spawned from a profiled one).
usage: mp_rank.py RANK UIDFILE [ITERS] [staged|sym|reg|rs|ag|ring|reforder] — rank 1 creates the ncclUniqueId and
writes it to UIDFILE; `sym` puts both buffers in a symmetric window, `reg` registers them with ncclCommRegister
(zero-copy kernels either way), `eager` leaves them unregistered with NCCL_AMD_EAGER_REGISTER=1; `push` is the staged
AllReduce with the push gather (NCCL_AMD_AG_PULL=0); `rs` / `ag` run ReduceScatter (S in, S/n out) / AllGather (S/n in,
S out) on the staged path; `ring` / `reforder` the AllReduce with NCCL_ALGO=RING / NCCL_AMD_REF_ORDER=1 at K = 32
reference parts."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nccl_amd  # noqa: E402


def main():
    rank, path = int(sys.argv[1]), sys.argv[2]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    if rank == 1:
        uid = nccl_amd.get_unique_id()
        with open(path + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(path + ".tmp", path)
    else:
        t0 = time.time()
        while not os.path.exists(path):
            if time.time() - t0 > 60:
                raise TimeoutError("no unique id")
            time.sleep(0.05)
        uid = open(path, "rb").read()
    mode = sys.argv[4] if len(sys.argv) > 4 else "staged"
    if mode == "ring":
        os.environ.update(NCCL_ALGO="RING", NCCL_AMD_REF_NCHANNELS="32")
    if mode == "reforder":
        os.environ.update(NCCL_AMD_REF_ORDER="1", NCCL_AMD_REF_NCHANNELS="32")
    # the staged kernel unless the mode says otherwise (eager zero-copy is the multi-process default since round 6)
    os.environ.update(NCCL_AMD_EAGER_REGISTER="1" if mode == "eager" else "0")
    if mode == "push":
        os.environ.update(NCCL_AMD_AG_PULL="0")
    n = int(os.environ.get("NRANKS", "2"))
    torch.cuda.set_device(0)
    comm = nccl_amd.Communicator.init(n, rank, uid)
    S = 256 << 20
    if mode == "sym":
        win_t = torch.empty(2 * S, dtype=torch.uint8, device="cuda")
        win = comm.register_window(win_t.data_ptr(), 2 * S)
        x = win_t[:S].view(torch.float32)
        y = win_t[S:].view(torch.float32)
        x.fill_(float(rank + 1))
    else:
        x = torch.full((S // 4,), float(rank + 1), device="cuda")
        y = torch.empty_like(x)
    if mode == "reg":
        regs = [comm.register_buffer(x.data_ptr(), S), comm.register_buffer(y.data_ptr(), S)]
    s = torch.cuda.current_stream()
    if mode == "ag":
        y = torch.empty(S // 4, dtype=torch.float32, device="cuda")
    blk = S // 4 // n  # elements of one rank block

    def one():
        if mode == "rs":
            comm.reduce_scatter_raw(x.data_ptr(), y.data_ptr(), blk, 7, 0, s.cuda_stream)
        elif mode == "ag":
            comm.all_gather_raw(x.data_ptr(), y.data_ptr(), blk, 7, s.cuda_stream)
        else:
            comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), S // 4, 7, 0, s.cuda_stream)
    for _ in range(2):
        one()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        one()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / max(iters, 1)
    total = float(n * (n + 1) // 2)
    if mode == "rs":
        ok = bool((y[:blk] == total).all())
    elif mode == "ag":
        ok = all(bool((y[r * blk:(r + 1) * blk] == float(r + 1)).all()) for r in range(n))
    else:
        ok = bool((y == total).all())
    print(f"rank {rank}: ok={ok} async={comm.async_error()} ms={ms:.4f}", flush=True)
    if mode == "sym":
        comm.deregister_window(win)
    if mode == "reg":
        for h in regs:
            comm.deregister_buffer(h)
    comm.destroy()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
