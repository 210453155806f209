"""Two ranks of one process on the one GPU (NCCL_MULTI_RANK_GPU_ENABLE): a 256 MiB fp32 AllReduce per rank with
pinned host send / receive buffers (host_staged.direct at N = 2) vs device buffers, under the channel settings in
the environment (NCCL_MAX_CTAS ...). One JSON line: ms per collective (max over ranks' streams), bitwise check."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
import torch  # noqa: E402

import nccl_amd  # noqa: E402

count = 64 << 20
torch.cuda.set_device(0)
comms = nccl_amd.Communicator.init_all([0, 0])
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
ins = [(torch.randint(-1024, 1025, (count,), dtype=torch.int32).float() / 256) for _ in range(2)]
want = ins[0] + ins[1]
res = {"env": {k: v for k, v in os.environ.items() if k.startswith("NCCL_MAX_CTAS") or k.startswith("NCCL_AMD_LINK")}}
for kind in ("host", "device"):
    if kind == "host":
        xs = [x.pin_memory() for x in ins]
        ys = [torch.zeros(count).pin_memory() for _ in range(2)]
    else:
        xs = [x.cuda() for x in ins]
        ys = [torch.zeros(count, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()

    def run():
        nccl_amd.group_start()
        for c, s, x, y in zip(comms, streams, xs, ys):
            c.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, s.cuda_stream)
        nccl_amd.group_end()

    for _ in range(2):
        run()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in streams]
    for (a, _), s in zip(ev, streams):
        a.record(s)
    it = 5
    for _ in range(it):
        run()
    for (_, b), s in zip(ev, streams):
        b.record(s)
    torch.cuda.synchronize()
    res[f"{kind}_ms"] = round(max(a.elapsed_time(b) for a, b in ev) / it, 3)
    res[f"{kind}_ok"] = all(torch.equal(y.cpu(), want) for y in ys)
    del xs, ys
print(json.dumps(res), flush=True)
for c in comms:
    c.destroy()
