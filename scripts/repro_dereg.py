"""Repro of the N=4 rehearsal stall (bench.py suite: registered part, then the staged tuning matrix's first
communicator): NPROC processes on the one GPU. Each: a main communicator, a 256 MiB AllReduce on ncclCommRegister'd
buffers, deregistration, then MODE-dependent: a new communicator's 256 MiB staged AllReduce. Prints per rank the
seconds each phase took and the async errors. usage: python scripts/repro_dereg.py NPROC MODE
MODE: bench (as bench.py), nodereg (skip deregistration), barrier (host barrier after deregistration)"""
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, n, uids, mode, q):
    os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "20000"
    import torch
    import torch.distributed as dist
    import nccl_amd
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29877")
    dist.init_process_group("gloo", rank=rank, world_size=n)
    t = {}
    t0 = time.perf_counter()
    comm = nccl_amd.Communicator.init(n, rank, uids[0])
    s = torch.cuda.current_stream()
    S = 256 << 20
    c = S // 4
    base = torch.randint(-1024, 1025, (c,), device="cuda", dtype=torch.int32).float() / 256
    sendr = base * (rank + 1)
    recvr = torch.empty_like(sendr)
    hs = [comm.register_buffer(sendr.data_ptr(), S), comm.register_buffer(recvr.data_ptr(), S)]
    for _ in range(5):
        comm.all_reduce_raw(sendr.data_ptr(), recvr.data_ptr(), c, 7, 0, s.cuda_stream)
    torch.cuda.synchronize()
    t["registered"] = round(time.perf_counter() - t0, 3)
    if mode != "nodereg":
        for h in hs:
            comm.deregister_buffer(h)
    del sendr, recvr, base
    if mode == "barrier":
        dist.barrier()
    t1 = time.perf_counter()
    xs = torch.empty(c, dtype=torch.float32, device="cuda").uniform_(-1, 1)
    ys = torch.empty_like(xs)
    cm = nccl_amd.Communicator.init(n, rank, uids[1])
    t["cm_init"] = round(time.perf_counter() - t1, 3)
    t2 = time.perf_counter()
    for _ in range(3):
        cm.all_reduce_raw(xs.data_ptr(), ys.data_ptr(), c, 7, 0, s.cuda_stream)
    torch.cuda.synchronize()
    t["cm_ar"] = round(time.perf_counter() - t2, 3)
    t["async"] = [comm.async_error(), cm.async_error()]
    cm.destroy()
    comm.destroy()
    q.put((rank, t))


if __name__ == "__main__":
    n, mode = int(sys.argv[1]), sys.argv[2]
    import nccl_amd
    uids = [nccl_amd.get_unique_id(), nccl_amd.get_unique_id()]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, uids, mode, q)) for r in range(n)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(n):
        r, t = q.get(timeout=240)
        res[r] = t
    for p in ps:
        p.join(timeout=60)
    print(mode, {r: res[r] for r in sorted(res)}, flush=True)
