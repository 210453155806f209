"""VERDICT r3 item 6, narrowed: the pipelined host-staged part of bench.py (two extra torch streams, events chained
across them and the launch stream, pinned copies on the extra streams) makes every later small collective of the
N = 2 one-GPU rehearsal take ~27.6 us instead of ~4 us. Each run applies ONE perturbation (STEP) between two
measurements of an 8-byte LL AllReduce on the launch stream (torch's current stream), on a fresh communicator:
  streams   create two torch streams (the stream pool) and use neither
  events    + record / wait events across them and the launch stream (no copies)
  events1   the same with ONE extra stream
  launch_other  one kernel on an extra stream, synchronized (no events, no copies)
  events_r0 "events" on rank 0 only (rank 1 keeps one queue)
  copies    + pinned H2D / D2H copies on them, no events
  pipe      bench.host_staged's pipelined step itself (streams, events, copies)
  pipe_sync the same, then torch.cuda.synchronize() and the extra streams' references dropped
Launch each rank as its own process (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT set), e.g. rank 0 under rocprofv3.
Prints one JSON line per rank: us per call before / after."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import nccl_amd  # noqa: E402
from bench import _time_ms, exchange_unique_id  # noqa: E402


def main():
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    step = os.environ.get("STEP", "pipe")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream
    small = torch.ones(4, dtype=torch.float16, device="cuda")
    res = torch.empty_like(small)

    def measure(tag):
        cm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
        us = _time_ms(lambda: cm.all_reduce_raw(small.data_ptr(), res.data_ptr(), 4, 6, 0, sp), stream, 200,
                      align=dist.barrier) * 1e3
        cm.destroy()
        return us

    out = {"rank": rank, "step": step, "before_us": round(measure("before"), 2)}
    comm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
    count = (16 << 20) // 4
    h_in = torch.ones(count, dtype=torch.float32).pin_memory()
    h_out = torch.empty(count, dtype=torch.float32, pin_memory=True)
    d_in = torch.empty(count, dtype=torch.float32, device="cuda")
    d_out = torch.empty_like(d_in)
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    if step == "events_r0" and rank == 0:  # the extra queues on rank 0's process only
        step = "events"
    if step in ("events", "events1", "launch_other", "copies", "pipe", "pipe_sync"):
        for _ in range(5):
            ev0, ev1, ev2 = torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event()
            if step == "events1":  # one extra stream only
                ev0.record(stream)
                s_in.wait_event(ev0)
                ev1.record(s_in)
                stream.wait_event(ev1)
            elif step == "launch_other":  # a kernel on an extra stream, nothing else
                with torch.cuda.stream(s_in):
                    d_in.add_(1.0)
                torch.cuda.synchronize()
            elif step == "events":
                ev0.record(stream)
                s_in.wait_event(ev0)
                ev1.record(s_in)
                stream.wait_event(ev1)
                comm.all_reduce_raw(d_in.data_ptr(), d_out.data_ptr(), count, 7, 0, sp)
                ev2.record(stream)
                s_out.wait_event(ev2)
                ev3 = torch.cuda.Event()
                ev3.record(s_out)
                stream.wait_event(ev3)
            elif step == "copies":
                with torch.cuda.stream(s_in):
                    d_in.copy_(h_in, non_blocking=True)
                with torch.cuda.stream(s_out):
                    h_out.copy_(d_out, non_blocking=True)
                torch.cuda.synchronize()
            else:
                ev0.record(stream)
                s_in.wait_event(ev0)
                with torch.cuda.stream(s_in):
                    d_in.copy_(h_in, non_blocking=True)
                    ev1.record(s_in)
                stream.wait_event(ev1)
                comm.all_reduce_raw(d_in.data_ptr(), d_out.data_ptr(), count, 7, 0, sp)
                ev2.record(stream)
                with torch.cuda.stream(s_out):
                    s_out.wait_event(ev2)
                    h_out.copy_(d_out, non_blocking=True)
                ev3 = torch.cuda.Event()
                ev3.record(s_out)
                stream.wait_event(ev3)
    torch.cuda.synchronize()
    if step == "pipe_sync":
        del s_in, s_out
    comm.destroy()
    out["after_us"] = round(measure("after"), 2)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
