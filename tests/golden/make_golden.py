#!/usr/bin/env python3
"""Generate tests/golden/*.npz — golden vectors from an INDEPENDENT numpy restatement of the
reference's reduction semantics (not the C oracle, which these fixtures pin).

Reference rules restated (NVIDIA/nccl 2.30.7):
  - ring fold order: AllReduce block c (c = i // chunk, chunk = alignUp(divUp(count,n), 16/sizeof(T)),
    src/device/all_reduce.h:38-66) folds ranks c+1, c+2, ..., c — and, for NCCL_ALGO=RING at full size, the
    reference's own channel parts and loops (ring_parts / ring_owners below); ReduceScatter block d folds d+1..d
    (reduce_scatter.h:34-55); Reduce folds root+1..root (reduce.h:34-52).
  - every hop rounds to T (the FIFO holds T); acc_new = f(pre(x_local), acc) (common_kernel.h:83-121)
  - Min/Max/Sum/Prod semantics of reduce_kernel.h; avg = PreMulSum(1/n) on floats, SumPostDiv on ints.
The reference itself cannot be built or imported here (CUDA-only), so these are
restatement vectors; the reference's own known-answer tests are checked in tests/test_oracle.py.

Run: python tests/golden/make_golden.py   (rewrites the .npz files next to this script)
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def bf16_round(f32: np.ndarray) -> np.ndarray:
    u = f32.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = np.isnan(f32)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


def reduce_pair(kind, dtype, a, b):
    """f(a, b) with a = pre'd local input, b = accumulator; arrays in storage representation."""
    if dtype == "bf16":
        x, y = bf16_to_f32(a), bf16_to_f32(b)
        r = {"sum": x + y, "prod": x * y, "min": np.fmin(x, y), "max": np.fmax(x, y)}[kind]
        return bf16_round(r.astype(np.float32))
    if dtype == "f16":
        x, y = a.view(np.float16).astype(np.float32), b.view(np.float16).astype(np.float32)
        r = {"sum": x + y, "prod": x * y, "min": np.fmin(x, y), "max": np.fmax(x, y)}[kind]
        return r.astype(np.float16).view(np.uint16)
    if kind == "sum":
        return a + b
    if kind == "prod":
        return a * b
    if kind == "min":
        return np.fmin(a, b) if a.dtype.kind == "f" else np.minimum(a, b)
    return np.fmax(a, b) if a.dtype.kind == "f" else np.maximum(a, b)


def pre(kind, dtype, x, n):
    if kind != "avg" or dtype in ("i32", "u8", "i8", "u32", "i64"):
        return x
    if dtype == "f32":
        return (x * np.float32(1.0 / n)).astype(np.float32)
    if dtype == "bf16":
        s = bf16_to_f32(bf16_round(np.array([1.0 / n], dtype=np.float32)))[0]
        return bf16_round(bf16_to_f32(x) * s)
    raise ValueError(dtype)


def post(kind, dtype, x, n):
    if kind != "avg" or dtype in ("f32", "bf16", "f16"):
        return x
    # exact big-integer arithmetic: |x| // n with the sign restored (truncation toward zero)
    q = [(-(-int(v) // n) if int(v) < 0 else int(v) // n) for v in x.tolist()]
    bits = 8 * x.dtype.itemsize
    return np.array([v % (1 << bits) for v in q], dtype=np.uint64).astype(x.dtype.newbyteorder("=")) \
        if x.dtype.kind == "u" else np.array([((v + (1 << (bits - 1))) % (1 << bits)) - (1 << (bits - 1))
                                               for v in q], dtype=x.dtype)


def fold(kind, dtype, ins, idx, first, n):
    base = "sum" if kind == "avg" else kind
    acc = pre(kind, dtype, ins[first][idx], n)
    for k in range(1, n):
        r = (first + k) % n
        acc = reduce_pair(base, dtype, pre(kind, dtype, ins[r][idx], n), acc)
    return post(kind, dtype, acc, n)


NCCL_DT = {"i8": 0, "u8": 1, "i32": 2, "u32": 3, "i64": 4, "f16": 6, "f32": 7, "bf16": 9}
NCCL_OP = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
ESIZE = {"i8": 1, "u8": 1, "i32": 4, "u32": 4, "i64": 8, "f16": 2, "f32": 4, "bf16": 2}


def gen_inputs(rng, dtype, n, count):
    if dtype == "f32":
        return [rng.uniform(-1, 1, count).astype(np.float32) for _ in range(n)]
    if dtype == "bf16":
        return [bf16_round(rng.uniform(-1, 1, count).astype(np.float32)) for _ in range(n)]
    if dtype == "f16":
        return [rng.uniform(-1, 1, count).astype(np.float16).view(np.uint16) for _ in range(n)]
    info = {"i8": np.int8, "u8": np.uint8, "i32": np.int32, "u32": np.uint32, "i64": np.int64}[dtype]
    ii = np.iinfo(info)
    out = []
    for _ in range(n):
        x = rng.integers(ii.min, ii.max, count, dtype=info, endpoint=True)
        x[1::97] = ii.min
        x[2::97] = ii.max
        out.append(x)
    return out


def allreduce(kind, dtype, ins):
    n, count = len(ins), ins[0].size
    epp = 16 // ESIZE[dtype]
    chunk = -(-count // n)
    chunk = -(-chunk // epp) * epp
    out = np.empty_like(ins[0])
    for c in range(n):
        lo, hi = c * chunk, min(count, (c + 1) * chunk)
        if lo >= hi:
            continue
        out[lo:hi] = fold(kind, dtype, ins, slice(lo, hi), (c + 1) % n, n)
    return out


def ring_parts(count, esize, n, nchannels, buffsize, proto="simple"):
    """The reference's RING AllReduce partition of one task on a communicator of `nchannels` channels under
    protocol `proto` ("simple", "ll", "ll128") with that protocol's buffer size (0 = its default), restated from
    src/enqueue.cc:2091-2097 (channel shrink: threads x threshold 512 x 64, 512 x 8n, 640 x 8 with tuning.cc
    :244-257, 589-593), :576-757 (continuous-byte-distribution over cells of 32 KiB of traffic, AllReduce moving
    2 bytes of traffic per byte, 8 under LL, :461/:658; the first channel's part sized to the traffic per channel)
    and :2222-2321 (chunk: buffsize / 8 x 4 in 512-byte grains, / 8 / 2 in 16-byte grains, / 8 / 16 x 15 in
    1920-byte grains): returns the element counts of the channel parts, in channel order, and the chunk."""
    default = {"ll": 8 * 512 * 8 * 16, "ll128": 120 * 640 * 8 * 8, "simple": 1 << 22}[proto]
    buffsize = buffsize or default
    threads, threshold = {"simple": (512, 64), "ll": (512, 8 * n), "ll128": (640, 8)}[proto]
    tpb = 8 if proto == "ll" else 2           # traffic bytes per AllReduce byte
    nbytes = count * esize
    nc = nchannels
    while nc > 1 and nbytes < nc * threads * threshold:
        nc -= 1
    cell = -(-(32768 // tpb) // 16) * 16      # 32 KiB minimum traffic per channel, in data bytes
    ncells = -(-nbytes // cell)
    per_channel = -(-(max(32768, tpb * nbytes) // nc) // 16) * 16
    per = -(-per_channel // (tpb * cell))     # cells of traffic per channel
    step = min(ncells, per)
    first = ncells if nchannels == 1 else min(ncells, per)
    mids, last = divmod(ncells - first, step)
    if (first > 0) + mids + (last > 0) > nchannels:
        mids = nchannels - 2
        step = (ncells - first) // (mids + 1)
        last = step + (ncells - first) % (mids + 1)
    if last == 0 and mids:
        last, mids = step, mids - 1
    cells = [first] + [step] * mids + ([last] if last else [])
    parts = [c * cell // esize for c in cells]
    parts[-1] -= ncells * cell // esize - count
    stepsize = buffsize // 8
    chunk_bytes, grain = {"simple": (stepsize * 4, 512), "ll": (stepsize // 2, 16),
                          "ll128": (stepsize // 16 * 15, 1920)}[proto]
    chunk = chunk_bytes // grain * (grain // esize)
    return parts, chunk


def ring_owners(count, esize, n, nchannels, buffsize, proto="simple"):
    """Ring position that finalises each element: inside each channel part, loops of n chunks; the last loop's
    chunk is re-cut to alignUp(divUp(rem, n), 16 / esize) (src/device/all_reduce.h:34-38)."""
    parts, chunk = ring_parts(count, esize, n, nchannels, buffsize, proto)
    epp = 16 // esize
    owner = np.empty(count, dtype=np.int64)
    base = 0
    for p in parts:
        for start in range(0, p, n * chunk):
            rem = p - start
            ck = chunk if rem >= n * chunk else -(-(-(-rem // n)) // epp) * epp
            j = np.arange(min(rem, n * chunk))
            owner[base + start: base + start + j.size] = j // ck
        base += p
    assert base == count
    return owner


def allreduce_ring(kind, dtype, ins, nchannels, buffsize, proto="simple"):
    n, count = len(ins), ins[0].size
    owner = ring_owners(count, ESIZE[dtype], n, nchannels, buffsize, proto)
    out = np.empty_like(ins[0])
    for c in range(n):
        idx = np.nonzero(owner == c)[0]
        if idx.size:
            out[idx] = fold(kind, dtype, ins, idx, (c + 1) % n, n)
    return out


def reducescatter(kind, dtype, ins):
    n = len(ins)
    rc = ins[0].size // n
    return [fold(kind, dtype, ins, slice(d * rc, (d + 1) * rc), (d + 1) % n, n) for d in range(n)]


def reduce_root(kind, dtype, ins, root):
    n = len(ins)
    return fold(kind, dtype, ins, slice(0, ins[0].size), (root + 1) % n, n)


CASES = [
    ("allreduce", "sum", "f32", 2, 4099), ("allreduce", "sum", "f32", 3, 4099), ("allreduce", "sum", "f32", 8, 1037),
    ("allreduce", "prod", "f32", 3, 999), ("allreduce", "max", "f32", 4, 999), ("allreduce", "min", "f32", 4, 999),
    ("allreduce", "avg", "f32", 4, 2000), ("allreduce", "sum", "bf16", 4, 3001), ("allreduce", "avg", "bf16", 3, 3001),
    ("allreduce", "sum", "f16", 3, 2049), ("allreduce", "max", "bf16", 8, 1000),
    ("allreduce", "sum", "i32", 5, 2000), ("allreduce", "min", "i32", 5, 2000), ("allreduce", "max", "i32", 5, 2000),
    ("allreduce", "avg", "i32", 5, 2000), ("allreduce", "sum", "u8", 3, 777), ("allreduce", "avg", "u8", 3, 777),
    ("allreduce", "min", "i8", 4, 777), ("allreduce", "prod", "i64", 2, 500), ("allreduce", "avg", "i64", 3, 500),
    ("reducescatter", "sum", "f32", 4, 4 * 1001), ("reducescatter", "sum", "bf16", 8, 8 * 301),
    ("reducescatter", "max", "u32", 2, 2 * 1000),
    ("reduce", "min", "i32", 8, 3000), ("reduce", "max", "i32", 8, 3000), ("reduce", "sum", "f32", 4, 3000),
]
# NCCL_ALGO=RING AllReduce in the reference's full-size partition: (op, dtype, n, count, channels, NCCL_BUFFSIZE);
# small buffer sizes give several channel parts and several loops (the last one re-cut) at fixture sizes
RING_CASES = [
    ("sum", "f32", 3, 20000, 4, 16384), ("sum", "bf16", 4, 50001, 8, 16384), ("sum", "f16", 2, 70000, 3, 32768),
    ("max", "f32", 5, 30011, 6, 8192), ("avg", "f32", 8, 40000, 5, 16384), ("sum", "i32", 3, 9000, 2, 8192),
    ("sum", "f32", 2, 120_000, 7, 65536),
]
# the same ring on the LL and LL128 partitions (protocol buffer sizes NCCL_LL_BUFFSIZE / NCCL_LL128_BUFFSIZE; 0 =
# the reference's default): several channel parts and loops each
RING_PROTO_CASES = [
    ("sum", "f32", 3, 20000, 4, 65536, "ll"), ("sum", "bf16", 4, 30001, 5, 32768, "ll"),
    ("sum", "f16", 5, 60000, 6, 65536, "ll128"), ("max", "f32", 2, 25013, 3, 131072, "ll128"),
    ("sum", "f32", 8, 3000, 64, 0, "ll"), ("sum", "bf16", 3, 200_000, 4, 0, "ll128"),
]


def main():
    rng = np.random.default_rng(20261015)
    for f in os.listdir(HERE):
        if f.endswith(".npz"):
            os.remove(os.path.join(HERE, f))
    for i, (coll, kind, dtype, n, count) in enumerate(CASES):
        ins = gen_inputs(rng, dtype, n, count)
        d = {"coll": coll, "dtype": NCCL_DT[dtype], "op": NCCL_OP[kind], "n": n}
        for r, x in enumerate(ins):
            d[f"in{r}"] = x
        name = f"{i:02d}_{coll}_{kind}_{dtype}_n{n}"
        if coll == "allreduce":
            d["out"] = allreduce(kind, dtype, ins)
        elif coll == "reducescatter":
            for r, o in enumerate(reducescatter(kind, dtype, ins)):
                d[f"out{r}"] = o
        else:
            root = 0 if kind == "min" else n // 2
            d["root"] = root
            d["out"] = reduce_root(kind, dtype, ins, root)
            name += f"_root{root}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    for j, (kind, dtype, n, count, nch, buffsize) in enumerate(RING_CASES):
        ins = gen_inputs(rng, dtype, n, count)
        d = {"coll": "allreduce_ring", "dtype": NCCL_DT[dtype], "op": NCCL_OP[kind], "n": n, "nchannels": nch,
             "buffsize": buffsize}
        for r, x in enumerate(ins):
            d[f"in{r}"] = x
        d["out"] = allreduce_ring(kind, dtype, ins, nch, buffsize)
        name = f"{len(CASES) + j:02d}_allreduce_ring_{kind}_{dtype}_n{n}_k{nch}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    base = len(CASES) + len(RING_CASES)
    for j, (kind, dtype, n, count, nch, buffsize, proto) in enumerate(RING_PROTO_CASES):
        ins = gen_inputs(rng, dtype, n, count)
        d = {"coll": "allreduce_ring", "dtype": NCCL_DT[dtype], "op": NCCL_OP[kind], "n": n, "nchannels": nch,
             "buffsize": buffsize, "proto": proto}
        for r, x in enumerate(ins):
            d[f"in{r}"] = x
        d["out"] = allreduce_ring(kind, dtype, ins, nch, buffsize, proto)
        name = f"{base + j:02d}_allreduce_ring_{proto}_{kind}_{dtype}_n{n}_k{nch}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    print(f"wrote {base + len(RING_PROTO_CASES)} fixtures to {HERE}")


if __name__ == "__main__":
    main()
