"""CPU tests of the oracle (oracle/nccl_oracle.c) against the reference's known-answer tests and the
committed golden fixtures (tests/golden/, produced by the independent numpy restatement in
tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_kat_allreduce_rank_values(built, n):
    # docs/examples/03_collectives/01_allreduce/c/main.cc:112-168 and python/allreduce.py:97-116 (also
    # 04_user_buffer_registration/01_allreduce/c/main.cc:112-166 and 05_symmetric_memory/01_allreduce/c/
    # main.cc:112-170 with 1M floats; GPU: test_gpu_windows.py::test_reference_examples_symmetric_and_registered):
    # every rank fills its buffer with its rank id; every element of the result is n(n-1)/2.
    count = 32 * 1024
    ins = [np.full(count, float(r), dtype=np.float32) for r in range(n)]
    out = oracle.all_reduce(ins, 7, 0)
    assert np.all(out == np.float32(n * (n - 1) / 2))
    # the C example only sets element 0 to the rank and zeroes the rest
    ins = [np.zeros(count, dtype=np.float32) for _ in range(n)]
    for r in range(n):
        ins[r][0] = r
    out = oracle.all_reduce(ins, 7, 0)
    assert out[0] == n * (n - 1) / 2 and not out[1:].any()


@pytest.mark.parametrize("n", [2, 4, 8])
def test_kat_allgather_segments(built, n):
    # docs/examples/05_symmetric_memory/02_allgather/c/main.cc:160-175: segment r holds value r
    count = 1000
    out = oracle.all_gather([np.full(count, float(r), dtype=np.float32) for r in range(n)])
    for r in range(n):
        assert np.all(out[r * count:(r + 1) * count] == r)


def test_op_mapping_matches_host_to_dev_red_op(built):
    # src/enqueue.cc:2517-2526: xormask = (signed ? signBit : 0) ^ (max ? allBits : 0)
    assert oracle.dev_op(3, 2, 8) == (oracle.DEV_MINMAX, 0x80000000)   # int32 min
    assert oracle.dev_op(2, 2, 8) == (oracle.DEV_MINMAX, 0x7FFFFFFF)   # int32 max
    assert oracle.dev_op(3, 3, 8) == (oracle.DEV_MINMAX, 0)            # uint32 min
    assert oracle.dev_op(2, 1, 8) == (oracle.DEV_MINMAX, 0xFF)         # uint8 max
    assert oracle.dev_op(2, 4, 8) == (oracle.DEV_MINMAX, 0x7FFFFFFFFFFFFFFF)
    assert oracle.dev_op(2, 7, 8) == (oracle.DEV_MINMAX, 0xFFFFFFFF)   # float max: isMinNotMax = (arg&1)==0
    # avg: ints -> SumPostDiv(n<<1 | signed), floats -> PreMulSum(1/n in T) (enqueue.cc:2527-2571)
    assert oracle.dev_op(4, 2, 8) == (oracle.DEV_SUMPOSTDIV, (8 << 1) | 1)
    assert oracle.dev_op(4, 3, 8) == (oracle.DEV_SUMPOSTDIV, 8 << 1)
    assert oracle.dev_op(4, 7, 8) == (oracle.DEV_PREMULSUM, np.float32(0.125).view(np.uint32))
    assert oracle.dev_op(4, 6, 4) == (oracle.DEV_PREMULSUM, np.float16(0.25).view(np.uint16))
    assert oracle.dev_op(4, 9, 2) == (oracle.DEV_PREMULSUM, 0x3F00)  # bf16 0.5


def _golden_files():
    if not os.path.isdir(GOLDEN):
        return []
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz"))


PROTOS = {"ll": oracle.PROTO_LL, "ll128": oracle.PROTO_LL128, "simple": oracle.PROTO_SIMPLE}


@pytest.mark.parametrize("fname", _golden_files())
def test_oracle_matches_golden(built, fname):
    z = np.load(os.path.join(GOLDEN, fname), allow_pickle=False)
    coll, dtype, op, n = str(z["coll"]), int(z["dtype"]), int(z["op"]), int(z["n"])
    ins = [z[f"in{r}"] for r in range(n)]
    if coll == "allreduce":
        got = [oracle.all_reduce(ins, dtype, op)]
        want = [z["out"]]
    elif coll == "allreduce_ring":  # NCCL_ALGO=RING at full size: the reference's channel parts and loops
        proto = PROTOS[str(z["proto"])] if "proto" in z.files else oracle.PROTO_SIMPLE
        got = [oracle.all_reduce_ring_nccl(ins, dtype, op, int(z["nchannels"]), int(z["buffsize"]), proto)]
        want = [z["out"]]
    elif coll == "reducescatter":
        got = oracle.reduce_scatter(ins, dtype, op)
        want = [z[f"out{r}"] for r in range(n)]
    else:
        got = [oracle.reduce(ins, dtype, op, int(z["root"]))]
        want = [z["out"]]
    for g, w in zip(got, want):
        assert g.dtype == w.dtype and np.array_equal(g, w), f"{fname}: oracle differs from golden"


def test_float_sum_within_bound_of_exact(built):
    # SURVEY §8c bound vs the exact (float64) sum, for the nccl_ubx-style random inputs
    rng = np.random.default_rng(42)
    for n in (2, 8):
        for dtype, npdt in ((7, np.float32), (6, np.float16)):
            ins = [rng.standard_normal(10000).astype(npdt) for _ in range(n)]
            raw = [x.view(np.uint16) if dtype == 6 else x for x in ins]
            out = oracle.all_reduce(raw, dtype, 0)
            of = oracle.to_f32(dtype, out).astype(np.float64)
            exact = np.sum([x.astype(np.float64) for x in ins], axis=0)
            bound = oracle.float_tolerance(dtype, raw, of)
            assert np.all(np.abs(of - exact) <= bound)


def test_dyadic_fp32_sum_is_exact(built):
    n = 8
    ins = [oracle.fill(7, 100 + r, 50000, kind=1) for r in range(n)]
    out = oracle.all_reduce(ins, 7, 0)
    exact = np.sum([x.astype(np.float64) for x in ins], axis=0)
    assert np.array_equal(out.astype(np.float64), exact)


def test_integer_semantics(built):
    n = 5
    rng = np.random.default_rng(7)
    ins = [rng.integers(-2**31, 2**31, 4000, dtype=np.int64).astype(np.int32) for _ in range(n)]
    s = oracle.all_reduce(ins, 2, 0)
    want = (np.sum([x.astype(np.int64) for x in ins], axis=0) + 2**31) % 2**32 - 2**31
    assert np.array_equal(s.astype(np.int64), want)
    assert np.array_equal(oracle.all_reduce(ins, 2, 3), np.min(ins, axis=0))
    assert np.array_equal(oracle.all_reduce(ins, 2, 2), np.max(ins, axis=0))
    u = [x.view(np.uint32) for x in ins]
    assert np.array_equal(oracle.all_reduce(u, 3, 3), np.min(u, axis=0))
    # integer avg: wrapped sum, truncated toward zero (reduce_kernel.h:936-966)
    avg = oracle.all_reduce(ins, 2, 4)
    wv = want
    assert np.array_equal(avg.astype(np.int64), np.trunc(wv / n).astype(np.int64))


def test_fold_order_is_ring_order(built):
    # AllReduce: element i of block c (c = i // chunk) folds ranks c+1, ..., c (all_reduce.h:43-66).
    # Float sums are not associative, so a crafted case distinguishes the order.
    n = 3
    big, small = np.float32(2 ** 24), np.float32(1.0)
    ins = [np.array([big, big, big, big] * 3, dtype=np.float32),
           np.array([small] * 12, dtype=np.float32),
           np.array([-big] * 12, dtype=np.float32)]
    out = oracle.all_reduce(ins, 7, 0)
    chunk = 4  # alignUp(divUp(12,3), 4)
    for i in range(12):
        c = i // chunk
        order = [(c + 1 + k) % n for k in range(n)]
        acc = np.float32(ins[order[0]][i])
        for r in order[1:]:
            acc = np.float32(ins[r][i] + acc)
        assert out[i] == acc


def test_cpu_baseline_equals_oracle(built):
    ins = [oracle.fill(7, r, 123457) for r in range(4)]
    out, used = oracle.cpu_allreduce_f32(ins, 2)
    assert used >= 1
    assert np.array_equal(out, oracle.all_reduce(ins, 7, 0))


def test_ring_partition_matches_golden_restatement(built):
    """The C oracle's RING partition (oracle_ring_nccl_plan_proto) against the independent numpy restatement of
    tests/golden/make_golden.py over a sweep of sizes, types, rank and channel counts, protocols (Simple, LL,
    LL128) and protocol buffer sizes; the parts tile [0, count) and every plan uses at most the communicator's
    channels."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    rng = np.random.default_rng(8)
    counts = [1, 3, 4096, 8191, 100_003, 1 << 20, 67_108_864, 536_870_912] + [int(x) for x in rng.integers(1, 1 << 27, 40)]
    for count in counts:
        for es in (1, 2, 4, 8):
            for n, k in ((2, 1), (2, 256), (3, 7), (8, 32), (8, 64), (4, 2), (5, 3)):
                for proto, buffs in (("simple", (0, 16384, 1 << 20)), ("ll", (0, 4096, 65536)),
                                     ("ll128", (0, 32768, 1 << 20))):
                    for buff in buffs:
                        nch, lo, mid, hi, chunk = oracle.ring_nccl_plan(count, es, n, k, buff, PROTOS[proto])
                        parts, ck = mg.ring_parts(count, es, n, k, buff, proto)
                        assert [lo] + [mid] * (nch - 2) + ([hi] if nch > 1 else []) == parts, (count, es, n, k, buff,
                                                                                               proto)
                        assert ck == chunk and 1 <= nch <= k and sum(parts) == count and min(parts) > 0
    # protocol-specific constants: LL's 4 KiB cells and 32 KiB chunk, LL128's 576000-byte chunk (1920-byte grains)
    assert oracle.ring_nccl_plan(4096, 4, 2, 1, 0, oracle.PROTO_LL)[4] * 4 == 32768
    assert oracle.ring_nccl_plan(4096, 4, 2, 1, 0, oracle.PROTO_LL128)[4] * 4 == 576000
    assert oracle.ring_nccl_plan(1 << 20, 4, 2, 64, 0, oracle.PROTO_LL)[1] % 1024 == 0
    with pytest.raises(ValueError):  # a chunk below one grain never advances
        oracle.ring_nccl_plan(4096, 4, 2, 1, 1024, oracle.PROTO_LL128)


def test_ring_order_is_the_one_loop_order_when_one_loop(built):
    """On one channel and one loop the reference's ring order is the one-loop order every other path uses;
    beyond that the finalising ring position moves (so float sums differ), while integer sums never do."""
    for dt, count in ((7, 1000), (9, 4099), (6, 30_000)):
        ins = [oracle.fill(dt, 50 + r, count) for r in range(3)]
        assert np.array_equal(oracle.all_reduce_ring_nccl(ins, dt, 0, 1), oracle.all_reduce(ins, dt, 0))
    ins = [oracle.fill(9, 70 + r, 300_000) for r in range(3)]  # bf16: every hop rounds
    a, b = oracle.all_reduce_ring_nccl(ins, 9, 0, 16, 16384), oracle.all_reduce(ins, 9, 0)
    assert not np.array_equal(a, b)
    fa, fb = oracle.to_f32(9, a), oracle.to_f32(9, b)
    exact = sum(oracle.to_f32(9, x).astype(np.float64) for x in ins)
    bound = oracle.float_tolerance(9, ins, fb)
    assert np.all(np.abs(fa - exact) <= bound) and np.all(np.abs(fb - exact) <= bound)
    ins = [oracle.fill(2, 90 + r, 300_000) for r in range(3)]
    assert np.array_equal(oracle.all_reduce_ring_nccl(ins, 2, 0, 16, 16384), oracle.all_reduce(ins, 2, 0))


def test_two_ranks_fold_order_never_matters(built):
    """At n = 2 every element folds red(pre(x_b), pre(x_a)) with {a, b} = {0, 1}, and Sum / Prod / Min / Max / avg
    are commutative bit for bit (IEEE add and multiply, the ordered min / max), so the default one-loop order and
    the reference's full-size ring partition give identical bits for every type: config C2 (fp32 Sum, 2 ranks)
    equals the reference's RING/SIMPLE result on any channel count, not just within the float bound."""
    for dt in (7, 9, 6, 10, 11, 8):
        for op in (0, 1, 2, 3, 4):
            ins = [oracle.fill(dt, 500 + 7 * dt + op + r, 200_003) for r in range(2)]
            a = oracle.all_reduce(ins, dt, op)
            for k, buff in ((1, 0), (7, 16384), (64, 65536)):
                b = oracle.all_reduce_ring_nccl(ins, dt, op, k, buff)
                assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), (dt, op, k, buff)
