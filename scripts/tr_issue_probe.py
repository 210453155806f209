"""The small-AllReduce timing of bench.py's suite, reduced step by step (run under torch.distributed.run, one rank
per process, all on cuda:0): STEP=0 a fresh comm timed alone; 1 + the headline comm's 256 MiB AllReduces first;
2 + the headline comm kept alive while a second comm is timed (bench.py's per-column communicators)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NCCL_AMD_KERNEL_LOG", f"/tmp/tr_issue_klog_{os.getpid()}.log")
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import nccl_amd  # noqa: E402
from bench import _time_ms, exchange_unique_id, host_staged  # noqa: E402


def main():
    n, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    out = {}
    comm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
    small = torch.ones(2048, dtype=torch.float16, device="cuda")
    res = torch.empty_like(small)
    out["fresh"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp), stream, 200,
                            align=dist.barrier) * 1e3
    big = torch.ones(64 << 20, device="cuda")
    bres = torch.empty_like(big)
    for _ in range(10):
        comm.all_reduce_raw(big.data_ptr(), bres.data_ptr(), big.numel(), 7, 0, sp)
    torch.cuda.synchronize()
    out["after_big"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp), stream,
                                200, align=dist.barrier) * 1e3
    cm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
    out["second_comm"] = _time_ms(lambda: cm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp), stream,
                                  200, align=dist.barrier) * 1e3
    out["first_comm_again"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp),
                                       stream, 200, align=dist.barrier) * 1e3
    # a pinned host <-> device round trip on the suite's stream (bench.py's host-staged part does one before the
    # suite), then the same small AllReduce on that stream and on a fresh stream
    host = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
    dbuf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    dbuf.copy_(host, non_blocking=True)
    host.copy_(dbuf, non_blocking=True)
    torch.cuda.synchronize()
    out["after_pinned_copy"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp),
                                        stream, 200, align=dist.barrier) * 1e3
    fresh = torch.cuda.Stream()
    out["after_pinned_copy_fresh_stream"] = _time_ms(
        lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, fresh.cuda_stream), fresh, 200,
        align=dist.barrier) * 1e3
    del host
    torch.cuda.synchronize()
    out["after_pinned_freed"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp),
                                         stream, 200, align=dist.barrier) * 1e3
    # bench.py's pipelined host-staged bucket: the launch stream waits on events of two other streams and they on
    # its events; then the same small AllReduce on the launch stream and on a stream that took no part
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    ev0, ev1, ev2 = torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event()
    ev0.record(stream)
    s_in.wait_event(ev0)
    with torch.cuda.stream(s_in):
        dbuf.add_(1)
        ev1.record(s_in)
    stream.wait_event(ev1)
    comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp)
    ev2.record(stream)
    s_out.wait_event(ev2)
    torch.cuda.synchronize()
    out["after_event_chain"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp),
                                        stream, 200, align=dist.barrier) * 1e3
    other = torch.cuda.Stream()
    out["after_event_chain_other_stream"] = _time_ms(
        lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, other.cuda_stream), other, 200,
        align=dist.barrier) * 1e3
    # bench.py's host-staged part itself (256 MiB pinned buckets, serial then pipelined), then the small AllReduce on
    # the launch stream, on another stream, and on a new communicator
    hs = host_staged(comm, n, 64 << 20, stream, dist)
    out["host_staged_ms"] = hs["ms_per_step"] / 1e3
    out["after_host_staged"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp),
                                        stream, 200, align=dist.barrier) * 1e3
    out["after_host_staged_other_stream"] = _time_ms(
        lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, other.cuda_stream), other, 200,
        align=dist.barrier) * 1e3
    c3 = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
    out["after_host_staged_new_comm"] = _time_ms(
        lambda: c3.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, other.cuda_stream), other, 200,
        align=dist.barrier) * 1e3
    out["after_host_staged_plain_kernel"] = _time_ms(lambda: res.add_(1), stream, 200) * 1e3
    c3.destroy()
    cm.destroy()
    out["after_destroy"] = _time_ms(lambda: comm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 2048, 6, 0, sp),
                                    stream, 200, align=dist.barrier) * 1e3
    print(json.dumps({"rank": rank, **{k: round(v, 2) for k, v in out.items()}}), flush=True)
    comm.destroy()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
