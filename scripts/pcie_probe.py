"""PCIe copy probe for the host-staged bucket (bench.py host_staged): pinned H2D alone, D2H alone, and both at
once on two streams, 256 MiB each, HIP events. Prints one JSON line. Run under HSA_ENABLE_SDMA=0 / 1 to compare
the DMA engines with the runtime's blit kernels."""
import json
import os

import torch

S = 256 << 20
h_in = torch.empty(S, dtype=torch.uint8, pin_memory=True)
h_out = torch.empty(S, dtype=torch.uint8, pin_memory=True)
d_in = torch.empty(S, dtype=torch.uint8, device="cuda")
d_out = torch.empty(S, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, it=5):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    m = torch.cuda.current_stream()
    e0.record(m)
    for _ in range(it):
        fn()
    e1.record(m)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def h2d():
    d_in.copy_(h_in, non_blocking=True)


def d2h():
    h_out.copy_(d_out, non_blocking=True)


def both():
    m = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(m)
    s1.wait_stream(m)
    s2.wait_stream(m)
    with torch.cuda.stream(s1):
        d_in.copy_(h_in, non_blocking=True)
    with torch.cuda.stream(s2):
        h_out.copy_(d_out, non_blocking=True)
    m.wait_stream(s1)
    m.wait_stream(s2)


r = {"sdma": os.environ.get("HSA_ENABLE_SDMA", "default")}
for name, fn in (("h2d", h2d), ("d2h", d2h), ("both", both)):
    ms = timed(fn)
    r[name + "_ms"] = round(ms, 3)
    r[name + "_GBps"] = round((2 if name == "both" else 1) * S / (ms * 1e-3) / 1e9, 1)
print(json.dumps(r), flush=True)
