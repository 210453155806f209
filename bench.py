#!/usr/bin/env python3
"""bench.py — device-resident ncclAllReduce bus bandwidth of the MI355X engine (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
         --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one ncclAllReduce(sum, fp32) of the per-rank buffer, inputs already resident in HBM.
Workload (BASELINE.json configs):
  N == 1: configs[0] — 64 MiB fp32, world_size 1 loopback (the reference's nranks==1 out-of-place copy,
          src/device/onerank.cu:52-56). busBW is 0 by definition at n=1, so `value` is the HBM rate
          2*S/t (read S + write S), as BASELINE.md §2 prescribes for this config.
  N >= 2: the metric's 256 MiB fp32 per rank (configs[1] at N=2). `value` = whole-job bus bytes / time
          = N * busBW, busBW = algBW * 2(n-1)/n (reference plugins/profiler/inspector/inspector.cc:1450-1492).
          Per-rank busBW (the nccl-tests figure) is printed as `busbw_GBps`.
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


def hbm_bytes_per_rank(coll: str, n: int, S: int) -> int:
    """Algorithmic local-HBM bytes per launch per rank of this engine."""
    if n == 1:
        return 2 * S
    if coll == "allreduce":
        return int(2 * S + 4 * (n - 1) * S / n)
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
    """(value, algBW, busBW) in GB/s for one AllReduce of S bytes per rank taking ms_per_step."""
    algbw = S / (ms_per_step * 1e-3) / 1e9
    busbw = algbw * bus_factor("allreduce", n)
    value = 2 * S / (ms_per_step * 1e-3) / 1e9 if n == 1 else n * busbw
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
    return p.parse_args(argv)


def cpu_baseline(n: int, count: int, budget_s: float):
    """Naive OpenMP host reduction of n synthetic buffers, bounded to ~budget_s."""
    import numpy as np
    import oracle
    rng = np.random.default_rng(0x5EED0000)
    bufs = [rng.random(count, dtype=np.float32) * 2 - 1 for _ in range(n)]
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
    return {"value": round((n + 1) * S / t / 1e9, 2), "unit": "GB/s (host bytes: n reads + 1 write)",
            "cores": int(used), "kind": "port",
            "sample": f"{len(times)} runs x {n} x {S // MIB} MiB fp32 host buffers, median; cpu '{model}'"}


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
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = world
    import torch
    import nccl_amd

    ndev = torch.cuda.device_count()
    dev = local % max(ndev, 1)
    torch.cuda.set_device(dev)
    dist = None
    if n > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        comm = nccl_amd.Communicator.init(n, rank, exchange_unique_id(dist, rank))
    else:
        comm = nccl_amd.Communicator.init_all([dev])[0]

    size_mib = args.size_mib or (64 if n == 1 else 256)
    S = size_mib * MIB
    count = S // 4
    workload = (f"ncclAllReduce sum fp32, {size_mib} MiB, world_size=1 loopback" if n == 1 else
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
    barrier()
    t1 = time.perf_counter()
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
    hbm_bytes = hbm_bytes_per_rank("allreduce", n, S)
    achieved = hbm_bytes / (gpu_ms * 1e-3) / 1e9
    wkey = f"allreduce_f32_{size_mib}MiB_n{n}"
    traffic = load_pmc(wkey)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
            "traffic_source": "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, bytes/launch)"
            if traffic else None,
            "kernel": "copyKernel<4>" if n == 1 else "collKernel<float,SUM,AR>",
            "algorithmic_bytes_per_launch": hbm_bytes, "kernel_avg_ms": round(gpu_ms, 5)}
    if n > 1:
        link_peak = (n - 1) * XGMI_LINK_GBPS_DIR
        roof["xgmi"] = {"busbw": round(busbw, 1), "peak": round(link_peak, 1), "unit": "GB/s",
                        "frac": round(busbw / link_peak, 4),
                        "peak_basis": f"{n - 1} links x {XGMI_LINK_GBPS_DIR} GB/s per direction (spec/2)"}

    extra = {}
    if n == 1 and not args.no_extra and rank == 0:
        # secondary: the metric's 256 MiB at n=1 (> Infinity Cache, so HBM-bound)
        big = 256 * MIB // 4
        s2 = torch.empty(big, dtype=torch.float32, device="cuda").uniform_(-1, 1)
        r2 = torch.empty_like(s2)
        for _ in range(5):
            comm.all_reduce_raw(s2.data_ptr(), r2.data_ptr(), big, 7, 0, stream.cuda_stream)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(20):
            comm.all_reduce_raw(s2.data_ptr(), r2.data_ptr(), big, 7, 0, stream.cuda_stream)
        b.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        extra["n1_256MiB_hbm_GBps"] = round(2 * 256 * MIB / (ms * 1e-3) / 1e9, 1)
        # hipMemcpyAsync D2D of the same 256 MiB (the reference's nranks==1 implementation)
        a.record(stream)
        for _ in range(20):
            r2.copy_(s2)
        b.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        extra["n1_256MiB_hipMemcpyD2D_GBps"] = round(2 * 256 * MIB / (ms * 1e-3) / 1e9, 1)
        del s2, r2

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(n, count, args.cpu_seconds)
        except Exception as e:  # the baseline is reported, never required
            cpu = {"value": None, "error": repr(e)}
    barrier()

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: uniform[-1,1) fp32 per rank generated on device (torch RNG)",
            "config": {"workload": workload, "collective": "ncclAllReduce", "op": "sum", "bytes_per_rank": S,
                       "count": count, "n_ranks": n, "out_of_place": True,
                       "value_definition": "HBM GB/s = 2S/t (n=1)" if n == 1 else "N x busBW (whole job)"},
            "algbw_GBps": round(algbw, 2), "busbw_GBps": round(busbw, 2),
            "roofline": roof, "cpu_baseline": cpu, "check": "pass" if ok else "FAIL", **extra,
        }
        print(json.dumps(line), flush=True)
    comm.destroy()
    if dist is not None:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
