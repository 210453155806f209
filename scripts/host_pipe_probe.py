"""Host-staged bucket pipelines (bench.py host_staged): 256 MiB fp32 from pinned host memory, one-rank
ncclAllReduce, back to pinned host memory. Variants: serial on one stream; 3 streams with the AllReduce on its own
stream (a); the AllReduce behind its chunk's H2D on the H2D stream (d); copies only, no AllReduce (c: isolates how
the runtime moves the chunks); chunk counts from HOST_PIPE_CHUNKS (default 4,16), modes from HOST_PIPE_MODES
(default a,d); the AllReduce on the pinned host buffers themselves (direct: the kernel crosses PCIe). One JSON
line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nccl_amd  # noqa: E402

count = 64 << 20
comm = nccl_amd.Communicator.init_all([0])[0]
h_in = (torch.randint(-1024, 1025, (count,), dtype=torch.int32).float() / 256).pin_memory()
h_out = torch.empty(count, dtype=torch.float32, pin_memory=True)
d_in = torch.empty(count, dtype=torch.float32, device="cuda")
d_out = torch.empty_like(d_in)
main = torch.cuda.current_stream()
s_in, s_out, s_ar = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()


def ar(lo, hi, st):
    comm.all_reduce_raw(d_in[lo:].data_ptr(), d_out[lo:].data_ptr(), hi - lo, 7, 0, st.cuda_stream)


def serial():
    d_in.copy_(h_in, non_blocking=True)
    ar(0, count, main)
    h_out.copy_(d_out, non_blocking=True)


def make(nch, mode):
    cc = count // nch
    ev_in = [torch.cuda.Event() for _ in range(nch)]
    ev_ar = [torch.cuda.Event() for _ in range(nch)]

    def run():
        for s in (s_in, s_out, s_ar):
            s.wait_stream(main)
        for k in range(nch):
            lo, hi = k * cc, (k + 1) * cc if k + 1 < nch else count
            with torch.cuda.stream(s_in):
                d_in[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                if mode == "d":
                    ar(lo, hi, s_in)
                    ev_ar[k].record(s_in)
                else:
                    ev_in[k].record(s_in)
            if mode == "c":  # D2H of the chunk just copied in, no AllReduce
                ev_ar[k] = ev_in[k]
            if mode == "a":
                s_ar.wait_event(ev_in[k])
                ar(lo, hi, s_ar)
                ev_ar[k].record(s_ar)
            s_out.wait_event(ev_ar[k])
            with torch.cuda.stream(s_out):
                h_out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)
        for s in (s_in, s_out, s_ar):
            main.wait_stream(s)
    return run


def timed(fn, it=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(it):
        fn()
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def kernel_direct():  # the collective's kernel reads and writes the pinned host buffers over PCIe, no copies
    comm.all_reduce_raw(h_in.data_ptr(), h_out.data_ptr(), count, 7, 0, main.cuda_stream)


r = {"serial_ms": round(timed(serial), 3)}
want = h_in.clone()
if os.environ.get("HOST_PIPE_DIRECT", "1") == "1":
    h_out.zero_()
    r["direct_ms"] = round(timed(kernel_direct), 3)
    r["direct_ok"] = bool(torch.equal(h_out, want))
chunks = [int(c) for c in os.environ.get("HOST_PIPE_CHUNKS", "4,16").split(",") if c]
modes = os.environ.get("HOST_PIPE_MODES", "a,d").split(",")
for nch in chunks:
    for mode in modes:
        h_out.zero_()
        ms = timed(make(nch, mode))
        ok = bool(torch.equal(h_out, want)) if mode != "c" else None
        r[f"{mode}{nch}_ms"] = round(ms, 3)
        r[f"{mode}{nch}_ok"] = ok
r["GBps_note"] = "bucket bytes / ms (256 MiB)"
print(json.dumps(r), flush=True)
comm.destroy()
