"""n=2 one-GPU rehearsal of the AllReduce rate per element type and operator (both ranks in one process,
ncclCommInitAll([0, 0])), 256 MiB per rank: bytes per second of buffer for uint8 / fp8 / fp32 (and others)
under Sum and Avg, staged (default) or registered (MODE=reg: ncclCommRegister'd buffers, zero-copy kernel).
Prints one JSON line per (dtype, op). Results checked bit-exact against rank-independent expectations is not
possible for every type here, so this script only times; tests/ hold the parity checks.
usage: MODE=staged|reg python3 scripts/dtype_rate.py [MIB] [ITERS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"

import torch  # noqa: E402

import nccl_amd  # noqa: E402

MIB = 1 << 20
CASES = [("f32", 7, 0), ("f32", 7, 4), ("u8", 1, 0), ("u8", 1, 4), ("i8", 0, 2), ("u8", 1, 1),
         ("e4m3", 10, 0), ("e4m3", 10, 4), ("e5m2", 11, 0), ("bf16", 9, 0), ("bf16", 9, 4), ("f16", 6, 0)]
SIZE = {7: 4, 1: 1, 0: 1, 10: 1, 11: 1, 9: 2, 6: 2}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    mode = os.environ.get("MODE", "staged")
    only = os.environ.get("ONLY")
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0])
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    S = mib * MIB
    bufs = [torch.empty(2 * S, dtype=torch.uint8, device="cuda") for _ in comms]
    for b in bufs:  # small finite values in every type's encoding: bytes 0x00..0x3f
        b.copy_(torch.randint(0, 64, (2 * S,), dtype=torch.uint8, device="cuda"))
    regs = [cm.register_buffer(b.data_ptr(), 2 * S) for cm, b in zip(comms, bufs)] if mode == "reg" else []
    torch.cuda.synchronize()
    for name, dt, op in CASES:
        if only and name not in only.split(","):
            continue
        c = S // SIZE[dt]

        def step():
            with nccl_amd.group():
                for cm, s, b in zip(comms, streams, bufs):
                    cm.all_reduce_raw(b.data_ptr(), b.data_ptr() + S, c, dt, op, s.cuda_stream)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in streams]
        for (a, _), s in zip(ev, streams):
            a.record(s)
        for _ in range(iters):
            step()
        for (_, e), s in zip(ev, streams):
            e.record(s)
        torch.cuda.synchronize()
        ms = max(a.elapsed_time(e) for a, e in ev) / iters
        err = [cm.async_error() for cm in comms]
        print(json.dumps({"mode": mode, "dtype": name, "op": {0: "sum", 1: "prod", 2: "max", 4: "avg"}[op],
                          "bytes_per_rank": S, "ms": round(ms, 4), "GBps_per_rank": round(S / (ms * 1e-3) / 1e9, 1),
                          "async": err}), flush=True)
    for cm, h in zip(comms, regs):
        cm.deregister_buffer(h)
    for cm in comms:
        cm.destroy()


if __name__ == "__main__":
    main()
