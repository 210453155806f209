"""Small-AllReduce cost with one process per rank (ncclCommInitRank over the fd-server / dma-buf transport) vs all
ranks in one process (ncclCommInitAll), on the one GPU: host issue time per call (no sync) and device time per call
(events around a loop). Tells a per-call host cost in the multi-process path apart from GPU scheduling of several
processes on one device. usage: python scripts/mp_issue_probe.py [N] [BYTES] [ITERS]"""
import json
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"


def _loop(comms, streams, bufs, count, iters):
    import torch
    import nccl_amd
    one = len(comms) > 1

    def step():
        if one:
            with nccl_amd.group():
                for c, s, (x, y) in zip(comms, streams, bufs):
                    c.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 6, 0, s.cuda_stream)
        else:
            c, s, (x, y) = comms[0], streams[0], bufs[0]
            c.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 6, 0, s.cuda_stream)
    for _ in range(50):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    t1 = time.perf_counter()
    e1.record(streams[0])
    torch.cuda.synchronize()
    return (t1 - t0) / iters * 1e6, e0.elapsed_time(e1) / iters * 1e3


def _rank(rank, n, uid, nbytes, iters, q):
    if os.environ.get("KLOG"):  # as bench.py sets it: every distinct kernel named once in a file
        os.environ["NCCL_AMD_KERNEL_LOG"] = f"/tmp/mp_issue_klog_{os.getpid()}.log"
    import torch
    import nccl_amd
    torch.cuda.set_device(0)
    c = nccl_amd.Communicator.init(n, rank, uid)
    if os.environ.get("BIG"):  # a large AllReduce first, as bench.py's headline does before its suite
        big = torch.ones(64 << 20, device="cuda")
        for _ in range(5):
            c.all_reduce_raw(big.data_ptr(), big.data_ptr(), big.numel(), 7, 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        del big
    # STREAM=default: torch's current stream (the legacy null stream, as bench.py's suite used it)
    s = torch.cuda.current_stream() if os.environ.get("STREAM") == "default" else torch.cuda.Stream()
    x = torch.ones(nbytes // 2, dtype=torch.float16, device="cuda")
    y = torch.empty_like(x)
    host, dev = _loop([c], [s], [(x, y)], nbytes // 2, iters)
    q.put((rank, host, dev))
    c.destroy()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    nbytes = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 500
    import torch
    import nccl_amd
    uid = nccl_amd.get_unique_id()
    only_mp = os.environ.get("ONLY_MP") == "1"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, n, uid, nbytes, iters, q)) for r in range(n)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    print(json.dumps({"mode": "multi_process", "stream": os.environ.get("STREAM", "own"), "klog": bool(os.environ.get("KLOG")),
                      "big": bool(os.environ.get("BIG")), "n": n, "bytes": nbytes,
                      "host_us_per_call": [round(h, 2) for _, h, _ in res],
                      "device_us_per_call": [round(d, 2) for _, _, d in res]}), flush=True)
    if only_mp:
        return
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0] * n)
    streams = [torch.cuda.Stream() for _ in range(n)]
    bufs = [(torch.ones(nbytes // 2, dtype=torch.float16, device="cuda"),
             torch.empty(nbytes // 2, dtype=torch.float16, device="cuda")) for _ in range(n)]
    host, dev = _loop(comms, streams, bufs, nbytes // 2, iters)
    print(json.dumps({"mode": "one_process_group", "n": n, "bytes": nbytes, "host_us_per_group": round(host, 2),
                      "device_us_per_group": round(dev, 2)}), flush=True)
    for c in comms:
        c.destroy()


if __name__ == "__main__":
    main()
