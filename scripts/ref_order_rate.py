"""One-GPU rehearsal of the AllReduce rate with the default direct kernel, the direct kernel on the reference's
ring partition (NCCL_AMD_REF_ORDER=1) and the ring (NCCL_ALGO=RING), all ranks in one process, 256 MiB per rank.
Every mode is timed in REPS (default 3) interleaved rounds, the mode order rotated per round (each round creates the
mode's communicators, times ITERS AllReduces and destroys them), so a 5 % difference is not lost in drift between
repetitions. Prints one JSON line per (n, dtype, mode): median, min and max over the rounds.
usage: python scripts/ref_order_rate.py [MIB] [ITERS]"""
import json
import statistics
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
import torch  # noqa: E402

import nccl_amd  # noqa: E402

# ref_order_k32 / ring_k32: the reference's K = 32 parts shared by several workgroups (refSub, the channel cap at its
# default); *_cap32: one workgroup per part (NCCL_MAX_CTAS = 32, round 3's only form); ref_order_k64: the default K
# (the channel cap clamped to the reference's MAXCHANNELS). MODES_SEL=a,b picks modes (a clean kernel trace).
MODES = {"direct": {}, "ref_order_k32": {"NCCL_AMD_REF_ORDER": "1", "NCCL_AMD_REF_NCHANNELS": "32"},
         "ref_order_k64": {"NCCL_AMD_REF_ORDER": "1"},
         "ref_order_cap32": {"NCCL_AMD_REF_ORDER": "1", "NCCL_MAX_CTAS": "32"},
         "ring_k32": {"NCCL_ALGO": "RING", "NCCL_AMD_REF_NCHANNELS": "32"},
         "ring_cap32": {"NCCL_ALGO": "RING", "NCCL_MAX_CTAS": "32"}}
if os.environ.get("MODES_SEL"):
    MODES = {k: MODES[k] for k in os.environ["MODES_SEL"].split(",")}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    torch.cuda.set_device(0)
    for n in [int(x) for x in os.environ.get("NS", "2,4").split(",")]:
        for dt, tdt, es in ((7, torch.float32, 4), (9, torch.bfloat16, 2)):
            count = (mib << 20) // es
            bufs = [(torch.empty(count, dtype=tdt, device="cuda").uniform_(-1, 1), torch.empty(count, dtype=tdt, device="cuda"))
                    for _ in range(n)]
            order = list(MODES.items())
            if os.environ.get("REVERSE"):
                order.reverse()
            reps = int(os.environ.get("REPS", "3"))
            times = {mode: [] for mode, _ in order}
            errors = {mode: [] for mode, _ in order}
            for rep in range(reps):
                for j in range(len(order)):
                    mode, env = order[(j + rep) % len(order)]
                    for k in ("NCCL_AMD_REF_ORDER", "NCCL_MAX_CTAS", "NCCL_ALGO", "NCCL_AMD_REF_NCHANNELS"):
                        os.environ.pop(k, None)
                    os.environ.update(env)
                    comms = nccl_amd.Communicator.init_all([0] * n)
                    streams = [torch.cuda.Stream() for _ in range(n)]

                    def step():
                        with nccl_amd.group():
                            for c, s, (x, y) in zip(comms, streams, bufs):
                                c.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, dt, 0, s.cuda_stream)
                    for _ in range(3):
                        step()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(iters):
                        step()
                    for s in streams:
                        torch.cuda.current_stream().wait_stream(s)
                    e1.record()
                    torch.cuda.synchronize()
                    times[mode].append(e0.elapsed_time(e1) / iters)
                    errors[mode] += [c.async_error() for c in comms if c.async_error()]
                    for c in comms:
                        c.destroy()
            for mode, _ in order:
                ms = statistics.median(times[mode])
                print(json.dumps({"n": n, "dtype": dt, "mode": mode, "ms": round(ms, 4),
                                  "ms_min": round(min(times[mode]), 4), "ms_max": round(max(times[mode]), 4),
                                  "reps": len(times[mode]),
                                  "GBps_per_rank": round((mib << 20) / (ms * 1e-3) / 1e9, 1),
                                  "async": errors[mode]}), flush=True)
            del bufs


if __name__ == "__main__":
    main()
