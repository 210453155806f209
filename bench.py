#!/usr/bin/env python3
"""bench.py — device-resident ncclAllReduce bus bandwidth of the MI355X engine (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one ncclAllReduce(sum, fp32) of the per-rank buffer, inputs already resident in HBM.
Workload (BASELINE.json metric: 256 MiB fp32 at 1/2/4/8 GPUs):
  N == 1: 256 MiB fp32, world_size 1 (the reference's nranks==1 out-of-place copy,
          src/device/onerank.cu:52-56). busBW is 0 by definition at n=1, so `value` is the HBM rate
          2*S/t (read S + write S), as BASELINE.md §2 prescribes; configs[0] (64 MiB) is reported beside.
  N >= 2: the metric's 256 MiB fp32 per rank (configs[1] at N=2). `value` = busBW, the metric's own figure:
          algBW * 2(n-1)/n with algBW = S / t (reference plugins/profiler/inspector/inspector.cc:1450-1492, the
          nccl-tests number; t is the max over ranks, so it is the slowest rank's). It equals `busbw_GBps`, and
          `roofline.frac` is this figure (per launch) over the link peak. The whole-job sum N * busBW is printed
          beside it as `busbw_sum_GBps`.
Harness collectives (unique-id broadcast, barrier, max-over-ranks) use torch.distributed over gloo;
the measured AllReduce is this repo's libnccl.so (no RCCL anywhere on the data path).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "all-reduce bus GB/s (device-resident), 256 MiB fp32, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
XGMI_LINK_GBPS_DIR = 76.8     # 153.6 GB/s per link (spec, bidirectional) / 2 — SURVEY §8d
MIB = 1 << 20


def bus_factor(coll: str, n: int) -> float:
    """busBW / algBW (reference inspector.cc:1450-1492)."""
    if coll == "allreduce":
        return 2.0 * (n - 1) / n
    if coll in ("reducescatter", "allgather"):
        return (n - 1) / n
    return 1.0


def hbm_bytes_per_rank(coll: str, n: int, S: int, pull_gather: bool = True) -> int:
    """Algorithmic local-HBM bytes per launch per rank of this engine. Staged AllReduce: the scatter
    reads (n-1)/n S and writes it into the owners' staging, the fold reads S/n + (n-1)/n S and writes S/n; the push
    gather writes n-1 copies of the block and reads (n-1)/n S back (2S + 4(n-1)/n S), the pull gather (default) writes
    ONE copy and reads the peers' over the links (3S + 2(n-1)/n S). PMC at n = 2/4/8: 1.004 / 1.002 / 1.005 x the
    pull model (profiles/pmc_traffic.json)."""
    if n == 1:
        return 2 * S
    if coll == "allreduce":
        return int(3 * S + 2 * (n - 1) * S / n) if pull_gather else int(2 * S + 4 * (n - 1) * S / n)
    if coll == "allreduce_zero_copy":
        # symKernel on the ranks' own buffers (eager / registered): my input's S/n read for my block, its (n-1)/n S read
        # by the peers, my block written (S/n) and read by the n-1 peers, the other parts written ((n-1)/n S):
        # S + (2n-1)/n S = 3S - S/n (PMC at n = 2: 2.502 S, profiles/pmc_traffic.json)
        return int(3 * S - S / n)
    raise ValueError(coll)


def exchange_unique_id(dist, rank: int) -> bytes:
    """Rank 0 creates the ncclUniqueId (starts the bootstrap root), every rank receives it (gloo)."""
    import nccl_amd
    obj = [nccl_amd.get_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def max_over_ranks(dist, values):
    """Element-wise MAX over ranks (the contract's max-over-ranks timing)."""
    import torch
    if dist is None:
        return [float(v) for v in values]
    t = torch.tensor(values, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t]


def rates(n: int, S: int, ms_per_step: float):
    """(value, algBW, busBW) in GB/s for one AllReduce of S bytes per rank taking ms_per_step. value = busBW at
    n >= 2 (the metric, inspector.cc:1450-1492); at n = 1 busBW is 0 by definition, so value = the HBM rate 2S/t."""
    algbw = S / (ms_per_step * 1e-3) / 1e9
    busbw = algbw * bus_factor("allreduce", n)
    value = 2 * S / (ms_per_step * 1e-3) / 1e9 if n == 1 else busbw
    return value, algbw, busbw


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--size-mib", type=int, default=0, help="override per-rank buffer size")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true", help="skip the secondary 256 MiB n=1 measurement")
    p.add_argument("--no-suite", action="store_true", help="N>1: skip BASELINE configs 3-5 + link probes")
    p.add_argument("--quick-suite", action="store_true", help="N>1: smaller suite (rehearsal on one GPU)")
    return p.parse_args(argv)


def _time_ms(fn, stream, iters: int, warmup: int = 3, align=None) -> float:
    """Average device time of `fn` over `iters` back-to-back calls on `stream`. With several processes, `align`
    (a host barrier) lines the ranks up and one more untimed call follows it: a collective completes on every
    rank together, so the first event fires after every rank has reached the loop — without it, the ranks' host
    skew (hundreds of us after a gloo exchange) is timed as if it were the collective's (28 us "per call" for
    4 KiB AllReduces that take 4.5 us)."""
    import torch
    # every rank's earlier kernels are done before any rank launches this measurement's (BENCH_NO_LINEUP=1 skips it:
    # the check that the library's co-residency cap alone keeps ranks sharing a GPU from stalling)
    if align is not None and not os.environ.get("BENCH_NO_LINEUP"):
        torch.cuda.synchronize()
        align()
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if align is not None:
        align()
        fn()
    a.record(stream)
    h0 = time.perf_counter()
    for _ in range(iters):
        fn()
    h1 = time.perf_counter()
    b.record(stream)
    torch.cuda.synchronize()
    if os.environ.get("BENCH_HOST_US"):  # diagnostics: host issue time per call next to the device time
        print(f"[time_ms] host {(h1 - h0) / iters * 1e6:.2f} us/call, device {a.elapsed_time(b) / iters * 1e3:.2f} "
              f"us/call", file=sys.stderr, flush=True)
    return a.elapsed_time(b) / iters


def run_suite(comm, n: int, rank: int, dist, stream, quick: bool = False, out: dict | None = None) -> dict:
    """The other BASELINE.json configs at this N (the driver runs bench.py on the 8-GPU node, so this is
    where they get measured): RS+AG bf16 1 GiB bucket (configs[2]), AllReduce fp16 8 B..256 MiB sweep,
    LL / one-shot / direct / ring / tree (configs[3]: the reference's ring vs tree), Reduce int32 min/max 128 MiB root 0 (configs[4]); each with a
    size-independent exactness check, plus xGMI peer-copy probes for the roofline denominator."""
    t_start = time.perf_counter()

    def trace(part):  # BENCH_TRACE=1: when each suite part starts (diagnostics for stalls), on stderr
        if os.environ.get("BENCH_TRACE"):
            print(f"[rank {rank}] suite +{time.perf_counter() - t_start:.2f}s {part}", file=sys.stderr, flush=True)

    import torch
    import nccl_amd
    out = {} if out is None else out  # filled as it goes: a watchdog can report the finished parts
    sp = stream.cuda_stream

    def agree(ok: bool) -> bool:
        t = torch.tensor([0 if ok else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t[0]) == 0

    def tmax(ms: float) -> float:
        return max_over_ranks(dist, [ms])[0]

    def _tm(fn, stream_, iters: int, warmup: int = 3) -> float:  # collectives: ranks aligned first (_time_ms)
        return _time_ms(fn, stream_, iters, warmup, align=dist.barrier)

    # BENCH_SUITE_PARTS=a,b (diagnostics): only these parts, in the suite's fixed order
    only = [x for x in os.environ.get("BENCH_SUITE_PARTS", "").split(",") if x]
    selected = lambda part: not only or part in only
    g = torch.Generator(device="cuda")

    if selected("rs_ag_bf16"):
        trace("rs_ag_bf16")
        # --- configs[2]: ZeRO bucket, bf16, 1 GiB ---
        bucket = (64 if quick else 1024) * MIB
        cnt = bucket // 2
        g.manual_seed(77)
        base = torch.randint(-4, 5, (cnt,), device="cuda", generator=g, dtype=torch.int32).to(torch.bfloat16)
        send = base * (rank + 1)
        shard = torch.empty(cnt // n, dtype=torch.bfloat16, device="cuda")
        full = torch.empty(cnt, dtype=torch.bfloat16, device="cuda")
        rs = lambda: comm.reduce_scatter_raw(send.data_ptr(), shard.data_ptr(), cnt // n, 9, 0, sp)
        ag = lambda: comm.all_gather_raw(shard.data_ptr(), full.data_ptr(), cnt // n, 9, sp)
        ms_rs = tmax(_tm(rs, stream, 10))
        ms_ag = tmax(_tm(ag, stream, 10))
        rs()
        ag()
        torch.cuda.synchronize()
        ok = bool(torch.equal(full, base * (n * (n + 1) // 2)))
        bw = lambda ms: round(bucket / (ms * 1e-3) / 1e9 * (n - 1) / n, 2)
        out["rs_ag_bf16"] = {"config": f"ncclReduceScatter + ncclAllGather bf16, {bucket // MIB} MiB bucket, n={n}",
                             "rs_ms": round(ms_rs, 4), "rs_busbw_GBps": bw(ms_rs), "ag_ms": round(ms_ag, 4),
                             "ag_busbw_GBps": bw(ms_ag), "check": "pass" if agree(ok) else "FAIL"}
        # the same with the pull variants of both phases (xGMI reads instead of writes), its own communicator
        pulls = ("NCCL_AMD_RS_PULL", "NCCL_AMD_AG_PULL")
        saved_p = {k: os.environ.get(k) for k in pulls}
        os.environ.update({k: "1" for k in pulls})
        cp = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
        for k, v in saved_p.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
        ms_rs = tmax(_tm(lambda: cp.reduce_scatter_raw(send.data_ptr(), shard.data_ptr(), cnt // n, 9, 0, sp), stream, 10))
        ms_ag = tmax(_tm(lambda: cp.all_gather_raw(shard.data_ptr(), full.data_ptr(), cnt // n, 9, sp), stream, 10))
        full.zero_()
        cp.reduce_scatter_raw(send.data_ptr(), shard.data_ptr(), cnt // n, 9, 0, sp)
        cp.all_gather_raw(shard.data_ptr(), full.data_ptr(), cnt // n, 9, sp)
        torch.cuda.synchronize()
        okp = bool(torch.equal(full, base * (n * (n + 1) // 2)))
        cp.destroy()
        out["rs_ag_bf16"]["pull"] = {"rs_ms": round(ms_rs, 4), "rs_busbw_GBps": bw(ms_rs), "ag_ms": round(ms_ag, 4),
                                     "ag_busbw_GBps": bw(ms_ag), "check": "pass" if agree(okp) else "FAIL",
                                     "env": "NCCL_AMD_RS_PULL=1 NCCL_AMD_AG_PULL=1"}
        del send, shard, full, base

    if selected("ar_fp16_sweep"):
        trace("ar_fp16_sweep")
        # --- configs[3]: fp16 AllReduce sweep: LL vs one-shot vs direct. Protocol/algorithm knobs are read at
        #     communicator init (like the reference's NCCL_PARAMs), so each column gets its own communicator ---
        top = (16 if quick else 256) * MIB
        # small integers (|x| <= 8 * n): every fp16 sum is exact in any fold order, so every column's result must
        # equal base * n(n+1)/2 bit for bit — the sweep checks LL / LL128 / one-shot / ring / tree over the links
        # (LL's 8-byte flag/data atomicity across devices) at every size it times
        g.manual_seed(555)
        base = torch.randint(-8, 9, (top // 2,), device="cuda", generator=g, dtype=torch.int32).to(torch.float16)
        buf = base * (rank + 1)
        want = base * (n * (n + 1) // 2)
        res = torch.empty_like(buf)
        sweep_check = {}
        cols = {"ll": {"NCCL_PROTO": "LL"}, "ll128": {"NCCL_PROTO": "LL128"},
                "oneshot": {"NCCL_ALGO": "ONESHOT", "NCCL_PROTO": "Simple"},
                "direct": {"NCCL_ALGO": "DIRECT", "NCCL_PROTO": "Simple"},
                "ring": {"NCCL_ALGO": "RING"}, "tree": {"NCCL_ALGO": "TREE"}, "default": {},
                # the reference's RING/SIMPLE partition walked by the direct kernel: its cost vs default
                "reforder": {"NCCL_AMD_REF_ORDER": "1"}}
        if os.environ.get("BENCH_SWEEP_COLS"):  # diagnostics: a subset of the columns
            cols = {k: cols[k] for k in os.environ["BENCH_SWEEP_COLS"].split(",")}
        limits = {"ll": 512 * 1024, "ll128": 896 * 1024, "oneshot": 64 * MIB}
        rows = {}
        saved = {k: os.environ.get(k) for k in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_AMD_NO_AGGREGATION", "NCCL_AMD_REF_ORDER")}
        for name, env in cols.items():  # ll128: the LL64-line protocol (64-byte lines)
            for k in saved:
                os.environ.pop(k, None)
            os.environ.update(env)
            cm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
            size = 8
            while size <= top:
                if size <= limits.get(name, top):
                    c = size // 2
                    it = 50 if size <= 4 * MIB else 10
                    res[:c].zero_()
                    ms = tmax(_tm(lambda: cm.all_reduce_raw(buf.data_ptr(), res.data_ptr(), c, 6, 0, sp), stream, it))
                    torch.cuda.synchronize()
                    if not torch.equal(res[:c], want[:c]) and name not in sweep_check:
                        sweep_check[name] = f"FAIL at {size} bytes"
                    row = rows.setdefault(size, {"bytes": size})
                    row[name + "_us"] = round(ms * 1e3, 2)
                    row[name + "_busbw_GBps"] = round(size / (ms * 1e-3) / 1e9 * bus_factor("allreduce", n), 2)
                size *= 2
            torch.cuda.synchronize()
            cm.destroy()
        out["ar_fp16_sweep"] = [rows[k] for k in sorted(rows)]
        out["ar_fp16_sweep_check"] = {name: ("pass (exact integer sums, every size)" if agree(name not in sweep_check)
                                             else sweep_check.get(name, "FAIL on another rank")) for name in cols}
        out["size_table_row"] = size_table_row(n, out["ar_fp16_sweep"])
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
        del buf, res, base, want

    if selected("group_aggregation"):
        trace("group_aggregation")
        # --- group aggregation: 32 small AllReduce ops in one ncclGroupStart/End,
        #     one LL launch vs one launch per op ---
        agg = {}
        g.manual_seed(556)  # small integers: exact sums, so both columns are checked against base * n(n+1)/2
        base = torch.randint(-8, 9, (32 * 4096,), device="cuda", generator=g, dtype=torch.int32).to(torch.float16)
        buf = base * (rank + 1)
        res = torch.empty_like(buf)
        okg = True
        saved = {k: os.environ.get(k) for k in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_AMD_NO_AGGREGATION", "NCCL_AMD_REF_ORDER")}
        for name, env in (("aggregated", {}), ("one_launch_per_op", {"NCCL_AMD_NO_AGGREGATION": "1"})):
            for k in saved:
                os.environ.pop(k, None)
            os.environ.update(env)
            cm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))

            def grouped():
                with nccl_amd.group():
                    for k in range(32):
                        cm.all_reduce_raw(buf.data_ptr() + k * 8192, res.data_ptr() + k * 8192, 2048, 6, 0, sp)
            res.zero_()
            ms = tmax(_tm(grouped, stream, 20))
            agg[name + "_us_per_group"] = round(ms * 1e3, 2)
            torch.cuda.synchronize()
            # op k reduces elements [4096 k, 4096 k + 2048) (4 KiB at an 8 KiB stride)
            okg = okg and bool(torch.equal(res.view(32, 4096)[:, :2048],
                                           (base * (n * (n + 1) // 2)).view(32, 4096)[:, :2048]))
            cm.destroy()
        agg["config"] = "32 x ncclAllReduce fp16 4 KiB in one group"
        agg["check"] = "pass (exact integer sums, both columns)" if agree(okg) else "FAIL"
        out["group_aggregation"] = agg
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
        del buf, res, base

    if selected("reduce_int32"):
        trace("reduce_int32")
        # --- configs[4]: Reduce int32 min / max, 128 MiB, root 0 ---
        S = (16 if quick else 128) * MIB
        c = S // 4
        g.manual_seed(99)
        base = torch.randint(-2**31 + 64, 2**31 - 64, (c,), device="cuda", generator=g, dtype=torch.int64).to(torch.int32)
        send = base + rank
        recv = torch.empty_like(send) if rank == 0 else None
        red = {}
        okr = True
        for name, op, want in (("min", 3, 0), ("max", 2, n - 1)):
            fn = lambda: comm.reduce_raw(send.data_ptr(), recv.data_ptr() if recv is not None else None, c, 2, op, 0, sp)
            ms = tmax(_tm(fn, stream, 10))
            fn()
            torch.cuda.synchronize()
            if rank == 0:
                okr = okr and bool(torch.equal(recv, base + want))
            red[name + "_ms"] = round(ms, 4)
            red[name + "_busbw_GBps"] = round(S / (ms * 1e-3) / 1e9, 2)
        red["config"] = f"ncclReduce min/max int32, {S // MIB} MiB, root 0, n={n}"
        red["check"] = "pass (bit-exact)" if agree(okr) else "FAIL"
        out["reduce_int32"] = red
        del send, recv, base

    if selected("symmetric_window"):
        trace("symmetric_window")
        # --- symmetric windows (zero-copy pull kernels): the headline AllReduce and the
        #     fp16 latency curve with send/recv inside an NCCL_WIN_COLL_SYMMETRIC window ---
        S = (16 if quick else 256) * MIB
        c = S // 4
        win_t = torch.empty(2 * S, dtype=torch.uint8, device="cuda")
        win = comm.register_window(win_t.data_ptr(), 2 * S)
        sendw = win_t[:S].view(torch.float32)
        recvw = win_t[S:].view(torch.float32)
        g.manual_seed(4321)
        base = torch.randint(-1024, 1025, (c,), device="cuda", generator=g, dtype=torch.int32).float() / 256
        sendw.copy_(base * (rank + 1))
        fn = lambda: comm.all_reduce_raw(sendw.data_ptr(), recvw.data_ptr(), c, 7, 0, sp)
        ms = tmax(_tm(fn, stream, 20, warmup=5))
        recvw.zero_()
        fn()
        torch.cuda.synchronize()
        oks = bool(torch.equal(recvw, base * (n * (n + 1) / 2)))
        sym = {"config": f"ncclAllReduce sum fp32, {S // MIB} MiB per rank, buffers in symmetric windows, n={n}",
               "ms": round(ms, 4), "busbw_GBps": round(S / (ms * 1e-3) / 1e9 * bus_factor("allreduce", n), 2),
               "value_equiv_GBps": round(n * S / (ms * 1e-3) / 1e9 * bus_factor("allreduce", n), 2),
               "check": "pass (dyadic, exact)" if agree(oks) else "FAIL"}
        lat = []
        hbuf = win_t[:S].view(torch.float16)
        hres = win_t[S:].view(torch.float16)
        g.manual_seed(557)  # small integers in the window: every size's result checked exactly
        hbase = torch.randint(-8, 9, (S // 2,), device="cuda", generator=g, dtype=torch.int32).to(torch.float16)
        hbuf.copy_(hbase * (rank + 1))
        hwant = hbase * (n * (n + 1) // 2)
        okw = True
        size = 8
        while size <= (16 if quick else 64) * MIB:
            cc = size // 2
            it = 50 if size <= 4 * MIB else 10
            hres[:cc].zero_()
            ms = tmax(_tm(lambda: comm.all_reduce_raw(hbuf.data_ptr(), hres.data_ptr(), cc, 6, 0, sp), stream, it))
            torch.cuda.synchronize()
            okw = okw and bool(torch.equal(hres[:cc], hwant[:cc]))
            lat.append({"bytes": size, "us": round(ms * 1e3, 2),
                        "busbw_GBps": round(size / (ms * 1e-3) / 1e9 * bus_factor("allreduce", n), 2)})
            size *= 4
        sym["ar_fp16_sweep"] = lat
        sym["ar_fp16_sweep_check"] = "pass (exact integer sums, every size)" if agree(okw) else "FAIL"
        del hbase, hwant
        out["symmetric_window"] = sym
        torch.cuda.synchronize()
        comm.deregister_window(win)
        del win_t, sendw, recvw, base, hbuf, hres

    if selected("staged_tuning"):
        trace("staged_tuning")
        # --- staged-path tuning matrix at the headline size (data for the next tuning round: knobs are read
        #     at communicator init, so each setting gets its own communicator, all created up front). The columns are
        #     timed in interleaved rounds (column order rotated per round) and reported as median / min / max over
        #     the rounds, so a 5 % effect is not lost in one column's drift between repetitions. Every column's result
        #     must equal the default column's bit for bit (same fold order), which checks the fence-free release over
        #     the links and the eager zero-copy kernel ---
        S = (16 if quick else 256) * MIB
        c = S // 4
        xs = torch.empty(c, dtype=torch.float32, device="cuda").uniform_(-1, 1)
        ys = torch.empty_like(xs)
        knobs = ("NCCL_AMD_SLOT_BYTES", "NCCL_AMD_NSLOTS", "NCCL_MAX_CTAS", "NCCL_AMD_MIN_CHANNEL_BYTES", "NCCL_AMD_AG_PULL",
                 "NCCL_AMD_RS_PULL", "NCCL_AMD_P2P_FENCE", "NCCL_AMD_EAGER_REGISTER")
        saved = {k: os.environ.get(k) for k in knobs}
        # (the staging slab is capped at 1 GiB per rank, so slot sizes scale with channels x slots x n:
        #  default 128 KiB slots at n = 8, 256 KiB with 128 channels)
        envs = [{}, {"NCCL_AMD_P2P_FENCE": "0"}, {"NCCL_AMD_P2P_FENCE": "1"}, {"NCCL_MAX_CTAS": "256"},
                {"NCCL_AMD_SLOT_BYTES": "32768"}, {"NCCL_AMD_SLOT_BYTES": "65536"},
                {"NCCL_AMD_NSLOTS": "3"}, {"NCCL_AMD_NSLOTS": "4"}, {"NCCL_MAX_CTAS": "128"},
                {"NCCL_MAX_CTAS": "64"}, {"NCCL_MAX_CTAS": "32"}, {"NCCL_AMD_MIN_CHANNEL_BYTES": "32768"},
                {"NCCL_AMD_AG_PULL": "0"}, {"NCCL_AMD_RS_PULL": "1"}, {"NCCL_AMD_AG_PULL": "0", "NCCL_AMD_RS_PULL": "1"},
                {"NCCL_AMD_EAGER_REGISTER": "1"}]
        if os.environ.get("BENCH_TUNING_COLS"):  # diagnostics: a subset of the columns, by index
            envs = [envs[int(i)] for i in os.environ["BENCH_TUNING_COLS"].split(",")]
        reps = int(os.environ.get("BENCH_TUNING_REPS", "3"))
        comms = []
        for env in envs:
            for k in knobs:
                os.environ.pop(k, None)
            # every column but the eager one tunes the staged kernel, whatever the caller's NCCL_AMD_EAGER_REGISTER
            # (eager zero-copy would otherwise take these collectives and no staged knob would matter)
            os.environ.update({"NCCL_AMD_EAGER_REGISTER": "0", **env})
            comms.append(nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank)))
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
        times = [[] for _ in envs]
        same = [True] * len(envs)
        errors = [None] * len(envs)
        ref = None
        for rep in range(reps):
            for j in range(len(envs)):
                i = (j + rep) % len(envs)
                cm = comms[i]
                trace(f"staged_tuning rep {rep} {envs[i] or 'default'}")
                ys.fill_(float("nan"))  # a launch that does no work (an aborted communicator) cannot pass the check
                ms = tmax(_tm(lambda: cm.all_reduce_raw(xs.data_ptr(), ys.data_ptr(), c, 7, 0, sp), stream, 10))
                torch.cuda.synchronize()
                times[i].append(ms)
                err = cm.async_error()
                if err:
                    errors[i] = errors[i] or f"async error {err} in round {rep}"
                    print(f"[rank {rank}] staged_tuning {envs[i] or 'default'} round {rep}: async error {err}",
                          file=sys.stderr, flush=True)
                if i == 0 and ref is None:
                    ref = ys.clone()
                elif ref is not None:
                    same[i] = same[i] and bool(torch.equal(ys, ref))
        tuning = []
        for i, env in enumerate(envs):
            med = statistics.median(times[i])
            tuning.append({"env": env or "default", "ms": round(med, 4), "ms_min": round(min(times[i]), 4),
                           "ms_max": round(max(times[i]), 4), "reps": len(times[i]),
                           "busbw_GBps": round(S / (med * 1e-3) / 1e9 * bus_factor("allreduce", n), 2),
                           "check": "pass (= default, bitwise)" if agree(same[i] and errors[i] is None) else
                                    f"FAIL ({errors[i] or 'results differ from the default column, or an async error on another rank'})"})
        torch.cuda.synchronize()
        for cm in comms:
            cm.destroy()
        out["staged_tuning"] = {"config": f"ncclAllReduce sum fp32, {S // MIB} MiB per rank, n={n}",
                                "method": f"{reps} interleaved rounds (column order rotated per round), 10 AllReduces "
                                          "per column per round, max over ranks; ms = median over rounds; every "
                                          "column but NCCL_AMD_EAGER_REGISTER=1 runs the staged kernel "
                                          "(NCCL_AMD_EAGER_REGISTER=0 added), 'default' = the staged defaults",
                                "runs": tuning}
        dflt = tuning[0] if not envs[0] else None
        eager = next((r for r in tuning if r["env"] == {"NCCL_AMD_EAGER_REGISTER": "1"}), None)
        if eager is not None:  # the unregistered buffers of the headline, registered on first use
            out["eager_zero_copy"] = {"env": "NCCL_AMD_EAGER_REGISTER=1", "ms": eager["ms"],
                                      "ms_min": eager["ms_min"], "ms_max": eager["ms_max"],
                                      "busbw_GBps": eager["busbw_GBps"],
                                      "staged_default_ms": dflt["ms"] if dflt else None, "check": eager["check"]}
        del xs, ys, ref

    if selected("xgmi_probe"):
        trace("xgmi_probe")
        # --- xGMI probes (rank 0, peer copies via hipMemcpyPeerAsync) ---
        ndev = torch.cuda.device_count()
        if rank == 0 and ndev > 1:
            try:  # never on the one-GPU rehearsal: a failure here is recorded, never costs the line
                probe = {}
                nbytes = 256 * MIB
                src = torch.empty(nbytes // 4, device="cuda:0")
                dsts = [torch.empty(nbytes // 4, device=f"cuda:{d}") for d in range(1, ndev)]
                ms = _time_ms(lambda: dsts[0].copy_(src), stream, 5)
                probe["one_link_0to1_GBps"] = round(nbytes / (ms * 1e-3) / 1e9, 1)
                streams = [torch.cuda.Stream(device=0) for _ in dsts]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(3):
                    for s, d in zip(streams, dsts):
                        with torch.cuda.stream(s):
                            d.copy_(src)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / 3
                probe["fanout_0toall_GBps"] = round(len(dsts) * nbytes / dt / 1e9, 1)
                probe["method"] = "torch copy_ (hipMemcpyPeerAsync); fan-out = concurrent copies on separate streams"
                # the CU-driven probe (tests/native/xgmi_probe): 16-byte vector loads/stores from GPU 0's CUs, the
                # access pattern of the collective kernels, one link and all links, write and read
                exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "native", "xgmi_probe")
                if os.path.exists(exe):
                    try:
                        import subprocess
                        r = subprocess.run([exe, "256", "10"], capture_output=True, text=True, timeout=120)
                        probe["cu_kernel"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                            {"error": f"rc {r.returncode}: {r.stderr.strip()[-200:]}"}
                    except Exception as e:
                        probe["cu_kernel"] = {"error": repr(e)}
                # single-copy atomicity over the link: GPU 1 writes LL-style lines into GPU 0's
                # uncached memory while GPU 0 polls them; torn 8/16/64/128-byte lines are counted (LL needs torn8 == 0,
                # an LL128-class protocol would need torn64 == torn128 == 0)
                exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "native", "store_atomicity_probe")
                if os.path.exists(exe):
                    try:
                        import subprocess
                        r = subprocess.run([exe, "1", "0", "20000", "64", "3000"], capture_output=True, text=True,
                                           timeout=60)
                        probe["store_atomicity"] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 \
                            else {"error": f"rc {r.returncode}: {r.stderr.strip()[-200:]}"}
                    except Exception as e:
                        probe["store_atomicity"] = {"error": repr(e)}
                out["xgmi_probe"] = probe
                del src, dsts
            except Exception as e:
                out["xgmi_probe"] = {"error": repr(e)}
        if dist is not None:
            dist.barrier()  # the other ranks wait here, not spinning in a collective, while rank 0 probes the links

    if selected("registered"):
        trace("registered")
        # --- buffers registered with ncclCommRegister (zero-copy kernel in registered mode): the
        #     headline AllReduce on plain torch allocations, no window. Last: the newest path, and its deregistration
        #     makes every peer release a mapping ---
        S = (16 if quick else 256) * MIB
        c = S // 4
        g.manual_seed(4322)
        base = torch.randint(-1024, 1025, (c,), device="cuda", generator=g, dtype=torch.int32).float() / 256
        sendr = base * (rank + 1)
        recvr = torch.empty_like(sendr)
        hs = [comm.register_buffer(sendr.data_ptr(), S), comm.register_buffer(recvr.data_ptr(), S)]
        fn = lambda: comm.all_reduce_raw(sendr.data_ptr(), recvr.data_ptr(), c, 7, 0, sp)
        ms = tmax(_tm(fn, stream, 20, warmup=5))
        recvr.zero_()
        fn()
        torch.cuda.synchronize()
        okr = bool(torch.equal(recvr, base * (n * (n + 1) / 2)))
        out["registered"] = {"config": f"ncclAllReduce sum fp32, {S // MIB} MiB per rank, ncclCommRegister'd buffers, n={n}",
                             "ms": round(ms, 4), "busbw_GBps": round(S / (ms * 1e-3) / 1e9 * bus_factor("allreduce", n), 2),
                             "check": "pass (dyadic, exact)" if agree(okr) else "FAIL"}
        torch.cuda.synchronize()
        for h in hs:
            comm.deregister_buffer(h)
        del sendr, recvr, base

    return out


def size_table_row(n: int, sweep: list) -> dict:
    """The crossovers this sweep measured, as an NCCL_AMD_SIZE_TABLE row: the largest size up to
    which LL beats one-shot and direct at every size, then the largest size above that up to which one-shot beats
    direct at every size (LL128 left to the built-in row). `file_line` can be adopted as is:
    NCCL_AMD_SIZE_TABLE=<file with that line>."""
    def last_win(col, others, above=0):
        if not any(col + "_us" in r for r in sweep):
            return None  # not measured: keep the built-in value
        lim = above
        for r in sweep:
            if r["bytes"] <= above:
                continue
            if col + "_us" not in r:
                break
            rivals = [r[o + "_us"] for o in others if o + "_us" in r]
            if rivals and r[col + "_us"] > min(rivals):
                break
            lim = r["bytes"]
        return lim
    ll = last_win("ll", ("oneshot", "direct"))
    one = last_win("oneshot", ("direct",), above=ll or 0)  # = ll: no one-shot range (direct right after LL)
    # 0 (the column never won) turns the range off; '-' (not measured) keeps the built-in value
    fmt = lambda b: "-" if b is None else (f"{b >> 20}M" if b and b % (1 << 20) == 0 else f"{b >> 10}K" if b and b % 1024 == 0 else str(b))
    return {"nranks": n, "ll_bytes": ll, "oneshot_bytes": one, "file_line": f"{n} {fmt(ll)} - {fmt(one)}",
            "method": "largest size of the fp16 sweep up to which the column is the fastest of LL / one-shot / direct "
                      "at every size (one-shot: vs direct); 0 = never, '-' = not measured (the built-in value)"}


def host_staged(comm, n: int, count: int, stream, dist) -> dict:
    """Buckets that start and end in pinned host memory: H2D copy + AllReduce + D2H copy per step."""
    import torch
    S = count * 4
    # dyadic values k/256: every sum is exact in any fold order, so the chunked bucket checks against the whole one
    h_in = (torch.randint(-1024, 1025, (count,), dtype=torch.int32).float() / 256).pin_memory()
    h_out = torch.empty(count, dtype=torch.float32, pin_memory=True)
    d_in = torch.empty(count, dtype=torch.float32, device="cuda")
    d_out = torch.empty_like(d_in)

    def step():
        d_in.copy_(h_in, non_blocking=True)
        comm.all_reduce_raw(d_in.data_ptr(), d_out.data_ptr(), count, 7, 0, stream.cuda_stream)
        h_out.copy_(d_out, non_blocking=True)

    ms = _time_ms(step, stream, 5, warmup=2)
    ms = max_over_ranks(dist, [ms])[0]
    ms_dev = _time_ms(lambda: comm.all_reduce_raw(d_in.data_ptr(), d_out.data_ptr(), count, 7, 0,
                                                  stream.cuda_stream), stream, 5, warmup=2)
    ms_dev = max_over_ranks(dist, [ms_dev])[0]
    # pipelined: the bucket in chunks over three streams — H2D of chunk k+1, the AllReduce of chunk k and the D2H
    # of chunk k-1 overlap, so both PCIe directions stay busy at once (the reference's proxy pipelines its
    # network-staged transfers the same way, src/proxy.cc:954-1012). 4 chunks 6.6 ms, 8 chunks 6.1-8.1 ms, 16 chunks
    # 9.4-17 ms (the runtime blocks inside some chunk copies' enqueue), 9.5 ms serial on the MI355X box
    if os.environ.get("BENCH_HOST_STAGED_PIPE") == "0":  # diagnostics: the one-stream measurement only
        return {"bytes_per_rank": S, "ms_per_step": round(ms, 4), "algbw_GBps_incl_pcie": round(S / (ms * 1e-3) / 1e9, 2),
                "device_resident_ms": round(ms_dev, 4)}
    # chunk counts timed in the same run: more chunks shorten the pipeline's fill and drain (one
    # chunk's H2D before the first AllReduce, one chunk's D2H after the last) but enqueue more copies
    s_in, s_out = torch.cuda.Stream(), torch.cuda.Stream()
    ev_start, ev_end = torch.cuda.Event(), torch.cuda.Event()

    def make_piped(nchunk):
        cc = count // nchunk
        ev_in = [torch.cuda.Event() for _ in range(nchunk)]
        ev_ar = [torch.cuda.Event() for _ in range(nchunk)]

        def piped():
            ev_start.record(stream)
            s_in.wait_event(ev_start)
            s_out.wait_event(ev_start)
            for k in range(nchunk):
                lo, hi = k * cc, (k + 1) * cc if k + 1 < nchunk else count
                with torch.cuda.stream(s_in):
                    d_in[lo:hi].copy_(h_in[lo:hi], non_blocking=True)
                    ev_in[k].record(s_in)
                stream.wait_event(ev_in[k])
                comm.all_reduce_raw(d_in[lo:].data_ptr(), d_out[lo:].data_ptr(), hi - lo, 7, 0, stream.cuda_stream)
                ev_ar[k].record(stream)
                with torch.cuda.stream(s_out):
                    s_out.wait_event(ev_ar[k])
                    h_out[lo:hi].copy_(d_out[lo:hi], non_blocking=True)
            ev_end.record(s_out)
            stream.wait_event(ev_end)
        return piped

    sweep = []
    for nchunk in (4, 8, 16):
        ms_p = _time_ms(make_piped(nchunk), stream, 5, warmup=2)
        sweep.append((nchunk, max_over_ranks(dist, [ms_p])[0]))
    torch.cuda.synchronize()
    ref = h_out.clone()  # the last pipelined bucket (16 chunks)
    step()
    torch.cuda.synchronize()
    same = bool(torch.equal(ref, h_out))  # ... equals the one-stream result bit for bit
    nchunk, ms_p = min(sweep, key=lambda t: t[1])
    # direct: the collective on the pinned host buffers themselves (the reference accepts any pointer the device can
    # reach, argcheck.cc:12-28) — its kernel reads and writes across PCIe, both directions at once, with no copies,
    # chunks or pipeline fill; the one-rank copy caps its grid for host buffers (NCCL_AMD_HOST_COPY_GRID)
    h_out.zero_()
    ms_d = _time_ms(lambda: comm.all_reduce_raw(h_in.data_ptr(), h_out.data_ptr(), count, 7, 0, stream.cuda_stream),
                    stream, 5, warmup=2)
    ms_d = max_over_ranks(dist, [ms_d])[0]
    torch.cuda.synchronize()
    same_d = bool(torch.equal(ref, h_out))
    # PCIe Gen5 x16 bound: 57 GB/s one direction, 96.5 GB/s both at once on the SDMA engines
    # (profiles/r03_host_staged_pipeline.json): S each way at 96.5 / 2 GB/s per direction. The direct kernel's
    # loads and stores exceed it (about 100 GB/s both ways at N = 1): the bound is the copy engines', not the link's
    bound_ms = S / (96.5e9 / 2) * 1e3
    return {"bytes_per_rank": S, "ms_per_step": round(ms, 4), "algbw_GBps_incl_pcie": round(S / (ms * 1e-3) / 1e9, 2),
            "device_resident_ms": round(ms_dev, 4),
            "method": "pinned hipMemcpyAsync H2D + ncclAllReduce + D2H on one stream, HIP events",
            "pipelined": {"chunks": nchunk, "ms_per_step": round(ms_p, 4),
                          "algbw_GBps_incl_pcie": round(S / (ms_p * 1e-3) / 1e9, 2),
                          "pcie_bound_ms": round(bound_ms, 3), "frac_of_pcie_bound": round(bound_ms / ms_p, 3),
                          "sweep_ms": {str(k): round(v, 4) for k, v in sweep},
                          "check": "pass" if same else "FAIL",
                          "method": "chunks timed at 4 / 8 / 16, the fastest reported: H2D stream, AllReduce on the "
                                    "launch stream, D2H stream, event-chained"},
            "direct": {"ms_per_step": round(ms_d, 4), "algbw_GBps_incl_pcie": round(S / (ms_d * 1e-3) / 1e9, 2),
                       "frac_of_pcie_bound": round(bound_ms / ms_d, 3), "speedup_vs_pipelined": round(ms_p / ms_d, 3),
                       "check": "pass" if same_d else "FAIL",
                       "method": "ncclAllReduce with the pinned host buffers as send and receive buffers, no copies"}}


def cpu_baseline(count: int, budget_s: float, nbuf: int = 8):
    """Naive host-core OpenMP element-wise sum of `nbuf` fp32 buffers of `count` elements (BASELINE.md §3:
    the same splitmix64 inputs as the oracle, the oracle's fold order), bounded to ~budget_s. The default
    nbuf = 8 is the 8-GPU node's reduction (one buffer per rank); GB/s over (nbuf + 1) * S host bytes."""
    import numpy as np
    import oracle
    bufs = [oracle.fill(7, 0x5EED0000 + r, count) for r in range(nbuf)]
    out, used = oracle.cpu_allreduce_f32(bufs)  # warm-up
    times = []
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < 3:
        t0 = time.perf_counter()
        out, used = oracle.cpu_allreduce_f32(bufs)
        times.append(time.perf_counter() - t0)
        if len(times) >= 200:
            break
    t = statistics.median(times)
    S = count * 4
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    del bufs, out
    return {"value": round((nbuf + 1) * S / t / 1e9, 2), "unit": f"GB/s (host bytes: {nbuf} reads + 1 write)",
            "cores": int(used), "kind": "port", "ms_per_reduction": round(t * 1e3, 3),
            "sample": f"{len(times)} runs of an OpenMP fp32 sum of {nbuf} x {S // MIB} MiB host buffers "
                      f"(splitmix64, oracle fold order), median; {used} threads; cpu '{model}'"}


def xgmi_denominator(n: int) -> dict | None:
    """Measured link rates (tests/native/xgmi_probe, rank 0, GPU 0 -> its peers) as the xGMI roofline
    denominator: n == 2 -> one link, unidirectional; n > 2 -> the fan-out to all peers scaled to n-1 links,
    capped by (n-1) single links. The collective's own store flavour (write-through stores into uncached
    staging) is measured beside the nontemporal rate and is what the kernel can reach."""
    exe = os.path.join(ROOT, "tests", "native", "xgmi_probe")
    if not os.path.exists(exe):
        return None
    import subprocess
    try:
        r = subprocess.run([exe, "256", "5"], capture_output=True, text=True, timeout=120)
        pr = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # a secondary measurement never costs the headline
        return {"error": repr(e)}
    if "error" in pr:
        return pr
    peers = pr["peers"]
    one = pr.get("wt_uncached_write_1link_GBps") or pr["write_1link_GBps"]
    fan = pr.get("wt_uncached_write_fanout_GBps") or pr["write_fanout_GBps"]
    peak = one if n == 2 else min((n - 1) * one, fan * (n - 1) / peers)
    return {"peak": round(peak, 1), "probe": pr,
            "peak_basis": ("measured: one link, write-through stores into uncached peer memory (the kernel's own "
                           "store flavour), GPU 0 -> GPU 1" if n == 2 else
                           f"measured: GPU 0's write-through fan-out to all {peers} peers x {n - 1}/{peers}, capped "
                           f"at {n - 1} x one link")}


def launched_kernels(path: str) -> list:
    """Kernels this process launched, in first-launch order (the library's NCCL_AMD_KERNEL_LOG: one line per
    distinct kernel and grid, "<demangled name> grid=<workgroups> block=<threads>")."""
    try:
        with open(path) as f:
            return [ln.rstrip("\n") for ln in f if ln.strip()]
    except OSError:
        return []


def load_pmc(workload_key: str):
    """HBM traffic per launch from the committed rocprofv3 PMC passes (profiles/), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            ent = json.load(f).get(workload_key)
            return None if ent is None else ent.get("bytes_per_launch")
    except (OSError, ValueError):
        return None


def main(argv=None):
    args = parse(argv)
    if os.environ.get("BENCH_STACKS_AFTER_S"):  # diagnostics: dump every thread's stack if the run stalls
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["BENCH_STACKS_AFTER_S"]), repeat=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = world
    # the library names every kernel it launches in this file (read before it loads): the roofline's kernel
    # comes from the run itself
    klog = os.environ.setdefault("NCCL_AMD_KERNEL_LOG", f"/tmp/nccl_amd_bench_kernels_{os.getpid()}.log")
    # warnings on stderr at least (the library is silent by default, as the reference is, and the GPU boxes export
    # NCCL_DEBUG=VERSION): a failing mapping check, a remap through hipIpc handles or a clamped knob is then on record
    # in the driver's log of a multi-GPU run
    if os.environ.get("NCCL_DEBUG", "").upper() in ("", "NONE", "VERSION"):
        os.environ["NCCL_DEBUG"] = "WARN"
    if os.path.exists(klog):
        os.remove(klog)
    import torch
    import nccl_amd

    ndev = torch.cuda.device_count()
    dev = local % max(ndev, 1)
    torch.cuda.set_device(dev)
    dist = None
    try:
        if n > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            comm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
        else:
            comm = nccl_amd.Communicator.init_all([dev])[0]
    except nccl_amd.NcclError as e:
        # e.g. the init-time mapping check failing on a new node: rank 0 still prints the line,
        # with no rate and the library's message, so the run says why instead of ending without output
        if rank == 0:
            print(json.dumps({
                "metric": METRIC, "value": 0.0, "unit": "GB/s", "n_gpus": n, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": None, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic", "config": {"workload": "ncclAllReduce sum fp32, 256 MiB per rank", "n_ranks": n},
                "check": "FAIL", "error": f"communicator init failed: {e} (every rank's NCCL WARN lines on stderr "
                                          "name what failed)"}), flush=True)
        return 1

    if os.path.exists(klog):  # init's own launches (the mapping check) are not the step's kernel
        os.remove(klog)
    size_mib = args.size_mib or 256
    S = size_mib * MIB
    count = S // 4
    workload = (f"ncclAllReduce sum fp32, {size_mib} MiB, world_size=1 (the metric's size at N=1)" if n == 1 else
                f"ncclAllReduce sum fp32, {size_mib} MiB per rank, {n}xMI355X direct scatter-reduce-gather")
    stream = torch.cuda.current_stream()
    send = torch.empty(count, dtype=torch.float32, device="cuda").uniform_(-1, 1)
    recv = torch.empty_like(send)

    def barrier():
        if dist is not None:
            dist.barrier()

    def step():
        comm.all_reduce_raw(send.data_ptr(), recv.data_ptr(), count, nccl_amd.DataType.FLOAT32, 0, stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()  # this rank's K steps are done; the MAX over ranks below covers the slowest
    barrier()
    wall = t1 - t0
    gpu_ms = e0.elapsed_time(e1) / args.steps
    wall, gpu_ms = max_over_ranks(dist, [wall, gpu_ms])
    err = comm.async_error()

    # size-independent correctness property at full size: dyadic inputs => exact sums
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    base = torch.randint(-1024, 1025, (count,), device="cuda", generator=g, dtype=torch.int32).float() / 256
    send.copy_(base * (rank + 1))
    step()
    torch.cuda.synchronize()
    want = base * (n * (n + 1) / 2)
    err2 = comm.async_error()
    ok = bool(torch.equal(recv, want)) and err == 0 and err2 == 0
    if not ok:
        bad = (recv != want).nonzero().flatten()
        print(f"[rank {rank}] CHECK FAILED: async errors {err}/{err2}, {bad.numel()} mismatches of {count}; "
              f"first idx {bad[:8].tolist()} got {recv[bad[:4]].tolist()} want {want[bad[:4]].tolist()}; "
              f"block size {count // n}", file=sys.stderr, flush=True)
    if dist is not None:
        t = torch.tensor([0 if ok else 1], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ok = int(t[0]) == 0

    ms_per_step = wall / args.steps * 1e3
    value, algbw, busbw = rates(n, S, ms_per_step)
    probe_links = n > 1 and torch.cuda.device_count() >= n  # ranks on separate GPUs: links exist to measure
    # the dominant (only) kernel of a step: the first one this process launched (warm-up of the same call)
    kernels = launched_kernels(klog)
    kname = kernels[0] if kernels else None
    zero_copy = bool(kname and "symKernel" in kname)  # eager zero-copy (NCCL_AMD_EAGER_REGISTER) or staged
    if n > 1 and zero_copy:
        workload = (f"ncclAllReduce sum fp32, {size_mib} MiB per rank, {n}xMI355X zero-copy (the ranks' buffers "
                    "registered on first use, DESIGN.md §10.3)")
    hbm_bytes = hbm_bytes_per_rank("allreduce_zero_copy" if zero_copy else "allreduce", n, S,
                                   pull_gather=os.environ.get("NCCL_AMD_AG_PULL", "1") != "0")
    # launch_avg_ms: HIP events on the launch stream around the K back-to-back launches of the timed loop / K
    # (one launch per step; the rocprofv3 kernel average in profiles/ is the cross-check)
    launch_ms = gpu_ms
    hbm_rate = hbm_bytes / (launch_ms * 1e-3) / 1e9
    wkey = f"allreduce_f32_{size_mib}MiB_n{n}" + ("_eager" if zero_copy else "")
    traffic = load_pmc(wkey)
    traffic_src = "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, bytes/launch)" if traffic else None
    if n == 1:
        roof = {"bound": "hbm", "achieved": round(hbm_rate, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(hbm_rate / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": kname, "launch_avg_ms": round(launch_ms, 5), "algorithmic_bytes_per_launch": hbm_bytes}
    else:
        # n >= 2: the binding roofline is the links (min(HBM, xGMI)); achieved = algorithmic
        # bus bytes per launch (2(n-1)/n x S per rank) / the launch time = busBW (inspector.cc:1450-1492)
        spec_peak = (n - 1) * XGMI_LINK_GBPS_DIR
        bus_rate = 2 * (n - 1) / n * S / (launch_ms * 1e-3) / 1e9
        meas = None
        # ranks on separate GPUs: a real xGMI measurement, taken while every rank waits at a host barrier
        # (no peer kernel spinning on its GPU or moving bytes over the links during the probe)
        probe = probe_links
        if probe:
            barrier()
        if rank == 0 and probe:
            meas = xgmi_denominator(n)
        if probe:
            barrier()
        if meas and "peak" in meas:
            peak, basis, pr = meas["peak"], meas["peak_basis"], meas["probe"]
        else:
            peak, pr = round(spec_peak, 1), None
            basis = ("spec/2: " + (f"{n - 1} links x {XGMI_LINK_GBPS_DIR} GB/s per direction" if probe else
                                   "the ranks share one GPU here, no link exists to measure") +
                     (f" ({meas['error']})" if meas and "error" in meas else ""))
        roof = {"bound": "xgmi", "achieved": round(bus_rate, 1), "peak": peak, "unit": "GB/s",
                "frac": round(bus_rate / peak, 4), "traffic": traffic, "traffic_source": traffic_src,
                "peak_basis": basis, "kernel": kname, "launch_avg_ms": round(launch_ms, 5),
                "algorithmic_bus_bytes_per_launch": int(2 * (n - 1) / n * S),
                "spec_peak": round(spec_peak, 1), "spec_frac": round(bus_rate / spec_peak, 4),
                "hbm": {"achieved": round(hbm_rate, 1), "peak": HBM_PEAK_GBPS, "frac": round(hbm_rate / HBM_PEAK_GBPS, 4),
                        "algorithmic_bytes_per_launch": hbm_bytes}}
        if pr is not None:
            roof["probe"] = pr

    extra = {}
    if n == 1 and not args.no_extra and rank == 0:
        # configs[0] (64 MiB loopback, fits the 256 MiB Infinity Cache) and hipMemcpyAsync D2D of the
        # headline size (the reference's own nranks==1 implementation, onerank.cu:52-56) side by side
        small = 64 * MIB // 4
        s2 = torch.empty(small, dtype=torch.float32, device="cuda").uniform_(-1, 1)
        r2 = torch.empty_like(s2)
        ms = _time_ms(lambda: comm.all_reduce_raw(s2.data_ptr(), r2.data_ptr(), small, 7, 0, stream.cuda_stream),
                      stream, 20, warmup=5)
        extra["n1_64MiB_hbm_GBps"] = round(2 * 64 * MIB / (ms * 1e-3) / 1e9, 1)
        del s2, r2
        ms = _time_ms(lambda: recv.copy_(send), stream, 20, warmup=5)
        extra[f"n1_{size_mib}MiB_hipMemcpyD2D_GBps"] = round(2 * S / (ms * 1e-3) / 1e9, 1)
        # cold-buffer rate: 4 input/output pairs rotated (2 GiB), so no input is still in the 256 MiB Infinity
        # Cache when it is read again — the headline loop re-reads one input, as nccl-tests does
        pairs = [(torch.empty(count, dtype=torch.float32, device="cuda").uniform_(-1, 1),
                  torch.empty(count, dtype=torch.float32, device="cuda")) for _ in range(4)]
        it = [0]

        def rotated():
            x, y = pairs[it[0] % 4]
            it[0] += 1
            comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, stream.cuda_stream)
        ms = _time_ms(rotated, stream, 40, warmup=8)
        cold = 2 * S / (ms * 1e-3) / 1e9
        extra[f"n1_{size_mib}MiB_rotated4_hbm_GBps"] = round(cold, 1)
        # the share of `frac` the 256 MiB Infinity Cache gives the re-read input: the same kernel on cold buffers
        roof["achieved_cold"] = round(cold, 1)
        roof["frac_cold"] = round(cold / HBM_PEAK_GBPS, 4)
        del pairs
    def run_host_staged():
        # host-staged bucket (the proxy/network-staged path analogue, reference src/proxy.cc:954-1012):
        # pinned host -> HBM, AllReduce, HBM -> pinned host, all on the launch stream
        try:
            extra["host_staged"] = host_staged(comm, n, count, stream, dist)
        except Exception as e:  # secondary measurement
            extra["host_staged"] = {"error": repr(e)}

    # Part order (the same at every N): the headline loop and its check, the link probe, the N = 1 extras and CPU
    # baseline, the suite (N > 1), then the host-staged bucket. Every collective-rate part runs on the launch stream alone; the
    # host-staged part is the only one that uses two more streams (its pipelined variant), i.e. two more hardware
    # queues per rank, which stay mapped for the rest of the process — so it runs after every part whose rate it
    # would change. Measured on the one-GPU rehearsal: once a rank process holds three or more hardware queues, every
    # later small collective takes ~27.6 us instead of ~4 us (profiles/r04_queue_order_n2_onegpu.txt).
    # BENCH_HOST_STAGED=first (diagnostics) runs it before the suite instead.
    if not args.no_extra and n > 1 and os.environ.get("BENCH_HOST_STAGED") == "first":
        run_host_staged()

    # the host-core baseline on rank 0 at every N (north_star: "in the same run"), while the other ranks wait at the
    # barrier below — it never overlaps a timed part of any rank
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(count, args.cpu_seconds)
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "error": repr(e)}
    barrier()

    def link_summary():
        """N > 1, top level: GPU 0's per-link rates (the roofline's probe) and the staged
        AllReduce with the release fence forced on / off (the suite's staged_tuning columns), each checked bitwise
        against the default column — the cross-device evidence that decides the fence default."""
        out = {}
        if n > 1:
            pr = roof.get("probe") or {}
            out["xgmi_links"] = ({"wt_uncached_write_per_link_GBps": pr.get("wt_uncached_write_per_link_GBps"),
                                  "read_per_link_GBps": pr.get("read_per_link_GBps"),
                                  "wt_uncached_write_fanout_GBps": pr.get("wt_uncached_write_fanout_GBps"),
                                  # the fan-out rate by workgroup count: what one channel sustains across the links,
                                  # the constant behind the n >= 3 CU budget (enqueue.cc linkChannelBudget)
                                  "wt_uncached_write_fanout_by_workgroups_GBps":
                                      pr.get("wt_uncached_write_fanout_by_workgroups_GBps"),
                                  "source": "tests/native/xgmi_probe on rank 0 (GPU 0 -> each peer GPU)"}
                                 if pr else {"skipped": "the ranks share one GPU: no link to measure"})
            runs = {json.dumps(r["env"], sort_keys=True): r for r in extra.get("suite", {}).get("staged_tuning", {}).get("runs", [])}
            on = runs.get(json.dumps({"NCCL_AMD_P2P_FENCE": "1"}, sort_keys=True))
            off = runs.get(json.dumps({"NCCL_AMD_P2P_FENCE": "0"}, sort_keys=True))
            dflt = runs.get(json.dumps("default"))
            out["p2p_fence"] = ({"fence_on_ms": on["ms"], "fence_off_ms": off["ms"], "default_ms": dflt["ms"] if dflt else None,
                                 "default_fence": "on" if probe_links else "off (every rank on one GPU)",
                                 "check": "pass" if on["check"].startswith("pass") and off["check"].startswith("pass")
                                 else "FAIL", "source": "suite.staged_tuning"}
                                if on and off else {"skipped": "suite not run"})
        return out

    def headline():
        return {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: uniform[-1,1) fp32 per rank generated on device (torch RNG)",
            "config": {"workload": workload, "collective": "ncclAllReduce", "op": "sum", "bytes_per_rank": S,
                       "count": count, "n_ranks": n, "out_of_place": True,
                       "value_definition": ("HBM GB/s = 2S/t (n=1: busBW = algBW x 2(n-1)/n is 0 by definition)"
                                            if n == 1 else "busBW = S/t x 2(n-1)/n, t = slowest rank (inspector.cc:"
                                            "1450-1492, the nccl-tests figure); busbw_sum_GBps = N x busBW")},
            "algbw_GBps": round(algbw, 2), "busbw_GBps": round(busbw, 2),
            **({"busbw_sum_GBps": round(n * busbw, 2)} if n > 1 else {}),
            "roofline": roof, "cpu_baseline": cpu, "check": "pass" if ok else "FAIL", **link_summary(), **extra,
        }

    if n > 1 and not args.no_suite:
        # The suite (secondary measurements) runs under a watchdog: if any part of it stalls, every rank
        # still ends and rank 0 still prints the headline line, with the parts that finished.
        import threading
        suite = {}
        extra["suite"] = suite
        done = threading.Event()
        limit = float(os.environ.get("BENCH_SUITE_TIMEOUT_S", "300"))
        t_suite = time.perf_counter()

        def watchdog():
            if done.wait(limit):
                return
            if rank == 0:
                extra["suite"] = dict(suite, error=f"suite stopped by the {limit:.0f} s watchdog; finished parts kept")
                try:
                    text = json.dumps(headline())
                except Exception:  # a part was being written at that instant: report the headline alone
                    extra["suite"] = {"error": f"suite stopped by the {limit:.0f} s watchdog"}
                    text = json.dumps(headline())
                print(text, flush=True)
            os._exit(0 if ok else 1)

        threading.Thread(target=watchdog, daemon=True).start()
        try:
            run_suite(comm, n, rank, dist, stream, quick=args.quick_suite, out=suite)
            torch.cuda.synchronize()
        except Exception as e:  # secondary measurements never fail the headline line
            # (a device error is sticky: report the headline with the parts that finished and leave at once; the
            # other ranks end through their watchdogs)
            suite["error"] = repr(e)[:600]
            suite["seconds"] = round(time.perf_counter() - t_suite, 1)
            done.set()
            if rank == 0:
                print(json.dumps(headline()), flush=True)
            os._exit(0 if ok else 1)
        barrier()
        done.set()
        suite["seconds"] = round(time.perf_counter() - t_suite, 1)
    if not args.no_extra and (n == 1 or os.environ.get("BENCH_HOST_STAGED") != "first"):
        run_host_staged()

    if rank == 0:
        print(json.dumps(headline()), flush=True)
    comm.destroy()
    if dist is not None:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
