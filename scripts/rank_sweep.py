"""One rank of an n-process configuration sweep on the one-GPU box (rendezvous through files, no launcher,
so rank 0 can run under rocprofv3 without any process being spawned from a profiled one).

usage: rank_sweep.py RANK NRANKS DIR [CONFIGS_JSON]
  CONFIGS_JSON: list of {"name": str, "env": {...}, "coll": "allreduce"|"rs"|"ag", "dtype": int,
                         "mib": per-rank MiB, "iters": int, "group": K (allreduce: K ops of mib/K in one group)}
Each config gets its own communicator (the engine reads its knobs at init). Rank 0 creates the unique id
of config k and writes DIR/uid_k; the others wait for it. Every rank times its own stream with HIP events
and appends one JSON line per config to DIR/rank<R>.jsonl; results are checked on dyadic / small-integer
inputs (exact sums) after the timed loop."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nccl_amd  # noqa: E402

MIB = 1 << 20
DEFAULT = [{"name": f"ar_f32_256MiB_ch{c}", "env": {"NCCL_MAX_CTAS": str(c)}, "coll": "allreduce", "dtype": 7,
            "mib": 256, "iters": 20} for c in (256, 128, 64, 32)]


def uid_for(rank, d, k):
    path = os.path.join(d, f"uid_{k}")
    if rank == 0:
        uid = nccl_amd.get_unique_id()
        with open(path + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(path + ".tmp", path)
        return uid
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > 120:
            raise TimeoutError(f"no unique id for config {k}")
        time.sleep(0.02)
    return open(path, "rb").read()


def main():
    rank, n, d = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    cfgs = json.loads(open(sys.argv[4]).read()) if len(sys.argv) > 4 else DEFAULT
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    out = open(os.path.join(d, f"rank{rank}.jsonl"), "a")
    base_env = dict(os.environ)
    for k, cfg in enumerate(cfgs):
        os.environ.clear()
        os.environ.update(base_env)
        os.environ.update(cfg.get("env", {}))
        comm = nccl_amd.Communicator.init(n, rank, uid_for(rank, d, k))
        coll, dt = cfg.get("coll", "allreduce"), cfg.get("dtype", 7)
        tdt = {7: torch.float32, 9: torch.bfloat16, 6: torch.float16, 2: torch.int32}[dt]
        S = int(cfg.get("mib", 256) * MIB)
        es = torch.tensor([], dtype=tdt).element_size()
        cnt = S // es
        g = torch.Generator(device="cuda")
        g.manual_seed(1000 + k)
        base = torch.randint(-64, 65, (cnt,), device="cuda", generator=g, dtype=torch.int32).to(tdt)
        if dt == 7:
            base = base / 256
        send = base * (rank + 1)
        K = int(cfg.get("group", 0))
        if coll == "allreduce" and K:  # one group of K AllReduces over K equal slices of the buffer
            recv = torch.empty_like(send)
            per = cnt // K

            def fn():
                with nccl_amd.group():
                    for i in range(K):
                        comm.all_reduce_raw(send.data_ptr() + i * per * es, recv.data_ptr() + i * per * es, per, dt,
                                            0, s.cuda_stream)
            want = lambda: base * (n * (n + 1) // 2)
        elif coll == "allreduce":
            recv = torch.empty_like(send)
            fn = lambda: comm.all_reduce_raw(send.data_ptr(), recv.data_ptr(), cnt, dt, 0, s.cuda_stream)
            want = lambda: base * (n * (n + 1) // 2)
        elif coll == "rs":
            recv = torch.empty(cnt // n, dtype=tdt, device="cuda")
            fn = lambda: comm.reduce_scatter_raw(send.data_ptr(), recv.data_ptr(), cnt // n, dt, 0, s.cuda_stream)
            want = lambda: (base * (n * (n + 1) // 2))[rank * (cnt // n):(rank + 1) * (cnt // n)]
        else:  # ag: sendcount = cnt // n
            recv = torch.empty(cnt, dtype=tdt, device="cuda")
            part = cnt // n
            send = (base[rank * part:(rank + 1) * part] * 1).contiguous()
            fn = lambda: comm.all_gather_raw(send.data_ptr(), recv.data_ptr(), part, dt, s.cuda_stream)
            want = lambda: base[:part * n]
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(cfg.get("iters", 20)):
                fn()
            b.record(s)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / cfg.get("iters", 20)
        recv.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            fn()
        torch.cuda.synchronize()
        ok = bool(torch.equal(recv, want())) and comm.async_error() == 0
        comm.destroy()
        line = {"name": cfg["name"], "rank": rank, "n": n, "coll": coll, "dtype": dt, "bytes_per_rank": S,
                "ms": round(ms, 5), "check": ok, "env": cfg.get("env", {})}
        out.write(json.dumps(line) + "\n")
        out.flush()
        print(json.dumps(line), flush=True)
        del send, recv, base
    return 0


if __name__ == "__main__":
    sys.exit(main())
