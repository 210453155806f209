"""GPU tests of the API semantics around the hot path: group deferral, custom PreMulSum operators
(host-immediate and device scalars), hipGraph capture/replay, ncclCommInitRank inside a group from one
thread, and failure detection (spin timeout -> async error, ncclCommAbort of a stuck collective).
All ranks share the box's single GPU (reference NCCL_MULTI_RANK_GPU_ENABLE, init.cc:68)."""
import ctypes
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture()
def two_comms(built):
    import torch
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0])
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    yield comms, streams
    for c in comms:
        if c.ptr:
            c.destroy()


def _inputs(n, count, seed=5):
    import oracle
    return [oracle.fill(7, seed + r, count) for r in range(n)]


def test_group_defers_launch_until_end(two_comms):
    import torch
    import nccl_amd
    import oracle
    comms, streams = two_comms
    count = 100_003
    ins = _inputs(2, count)
    sends = [torch.from_numpy(x).cuda() for x in ins]
    recvs = [torch.zeros(count, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    nccl_amd.group_start()
    for c, s, x, y in zip(comms, streams, sends, recvs):
        c.allreduce(x, y, nccl_amd.SUM, stream=s)
    torch.cuda.synchronize()
    assert not recvs[0].any() and not recvs[1].any(), "work started before ncclGroupEnd"
    nccl_amd.group_end()
    torch.cuda.synchronize()
    want = oracle.all_reduce(ins, 7, 0)
    for r, y in enumerate(recvs):
        got = y.cpu().numpy()
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (f"rank {r}: {bad.size} mismatches, first {bad[:6].tolist()}, "
                               f"got {got[bad[:4]].tolist()} want {want[bad[:4]].tolist()}, "
                               f"async {[c.async_error() for c in comms]}")


def test_group_of_mixed_collectives(two_comms):
    import torch
    import nccl_amd
    import oracle
    comms, streams = two_comms
    n, count = 2, 65_536
    ins = _inputs(n, count, seed=9)
    sends = [torch.from_numpy(x).cuda() for x in ins]
    ar = [torch.empty(count, device="cuda") for _ in range(n)]
    rs = [torch.empty(count // n, device="cuda") for _ in range(n)]
    ag = [torch.empty(count * n, device="cuda") for _ in range(n)]
    mx = [torch.empty(count, device="cuda") for _ in range(n)]
    torch.cuda.synchronize()
    with nccl_amd.group():
        for r in range(n):
            comms[r].allreduce(sends[r], ar[r], nccl_amd.SUM, stream=streams[r])
            comms[r].reduce_scatter(sends[r], rs[r], nccl_amd.SUM, stream=streams[r])
            comms[r].allgather(sends[r], ag[r], stream=streams[r])
            comms[r].reduce(sends[r], mx[r], nccl_amd.MAX, root=1, stream=streams[r])
    torch.cuda.synchronize()
    assert np.array_equal(ar[0].cpu().numpy(), oracle.all_reduce(ins, 7, 0))
    want_rs = oracle.reduce_scatter(ins, 7, 0)
    for r in range(n):
        assert np.array_equal(rs[r].cpu().numpy(), want_rs[r])
        assert np.array_equal(ag[r].cpu().numpy(), np.concatenate(ins))
    assert np.array_equal(mx[1].cpu().numpy(), oracle.reduce(ins, 7, 2, 1))


@pytest.mark.parametrize("count", [1_000, 50_001])  # LL protocol / one-shot
@pytest.mark.parametrize("device_scalar", [False, True])
def test_premulsum_custom_op(two_comms, device_scalar, count):
    import torch
    import nccl_amd
    import oracle
    comms, streams = two_comms
    ins = _inputs(2, count, seed=13)
    scal = np.float32(0.375)
    dev_scal = torch.tensor([scal], device="cuda")
    ops = [c.create_pre_mul_sum(float(scal), 7, dev_scal.data_ptr() if device_scalar else None) for c in comms]
    sends = [torch.from_numpy(x).cuda() for x in ins]
    recvs = [torch.empty(count, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    with nccl_amd.group():
        for c, s, x, y, op in zip(comms, streams, sends, recvs, ops):
            c.allreduce(x, y, op, stream=s)
    torch.cuda.synchronize()
    want = oracle.all_reduce(ins, 7, premul_scalar_bits=int(scal.view(np.uint32)))
    for y in recvs:
        assert np.array_equal(y.cpu().numpy(), want)
    for c, op in zip(comms, ops):
        c.destroy_op(op)
    with pytest.raises(nccl_amd.NcclError):
        comms[0].destroy_op(ops[0])


def test_hipgraph_capture_and_replay(two_comms):
    import torch
    import nccl_amd
    import oracle
    comms, _ = two_comms
    # replayed graphs run on the replay stream: give each rank a hardware queue of its own
    streams = [nccl_amd.dedicated_stream(0), nccl_amd.dedicated_stream(0)]
    count = 1 << 20
    x = [torch.empty(count, device="cuda") for _ in range(2)]
    y = [torch.empty(count, device="cuda") for _ in range(2)]
    graphs = [torch.cuda.CUDAGraph() for _ in range(2)]
    torch.cuda.synchronize()
    for r in range(2):  # capture each rank's collective on its own stream (launches never block)
        with torch.cuda.graph(graphs[r], stream=streams[r]):
            comms[r].all_reduce_raw(x[r].data_ptr(), y[r].data_ptr(), count, 7, 0, streams[r].cuda_stream)
    for it in range(3):
        ins = _inputs(2, count, seed=100 + it)
        for r in range(2):
            x[r].copy_(torch.from_numpy(ins[r]))
        torch.cuda.synchronize()
        for r in range(2):  # replay each rank's graph on its own stream (both must run concurrently)
            with torch.cuda.stream(streams[r]):
                graphs[r].replay()
        torch.cuda.synchronize()
        want = oracle.all_reduce(ins, 7, 0)
        for r in range(2):
            assert np.array_equal(y[r].cpu().numpy(), want), f"replay {it} rank {r}"


def test_hipgraph_mixed_sequence(two_comms):
    """One captured graph per rank holding a sequence that crosses every protocol — LL AllReduce,
    ReduceScatter, AllGather and Reduce, a one-shot and a direct AllReduce, a direct ReduceScatter —
    replayed with fresh inputs: every epoch, credit and LL flag lives in device memory, so each replay must
    continue the counters where the previous one left them (fp32 sums, bit-exact vs the oracle)."""
    import torch
    import nccl_amd
    import oracle
    comms, _ = two_comms
    streams = [nccl_amd.dedicated_stream(0), nccl_amd.dedicated_stream(0)]
    # (collective, input count per rank)
    seq = [("allreduce", 1000), ("reducescatter", 2 * 1024), ("allgather", 1536), ("reduce", 3000),
           ("allreduce", 100_000), ("allreduce", 1 << 20), ("reducescatter", 2 * (1 << 19))]
    outc = {"allreduce": lambda c: c, "reducescatter": lambda c: c // 2, "allgather": lambda c: 2 * c,
            "reduce": lambda c: c}
    xs = [[torch.empty(c, device="cuda") for _, c in seq] for _ in range(2)]
    ys = [[torch.empty(outc[k](c), device="cuda") for k, c in seq] for _ in range(2)]
    graphs = [torch.cuda.CUDAGraph() for _ in range(2)]
    torch.cuda.synchronize()
    for r in range(2):
        with torch.cuda.graph(graphs[r], stream=streams[r]):
            sp = streams[r].cuda_stream
            for (k, c), x, y in zip(seq, xs[r], ys[r]):
                if k == "allreduce":
                    comms[r].all_reduce_raw(x.data_ptr(), y.data_ptr(), c, 7, 0, sp)
                elif k == "reducescatter":
                    comms[r].reduce_scatter_raw(x.data_ptr(), y.data_ptr(), c // 2, 7, 0, sp)
                elif k == "allgather":
                    comms[r].all_gather_raw(x.data_ptr(), y.data_ptr(), c, 7, sp)
                else:
                    comms[r].reduce_raw(x.data_ptr(), y.data_ptr(), c, 7, 0, 1, sp)
    for it in range(4):
        ins = [_inputs(2, c, seed=300 + 10 * it + j) for j, (_, c) in enumerate(seq)]
        for r in range(2):
            for j in range(len(seq)):
                xs[r][j].copy_(torch.from_numpy(ins[j][r]))
        torch.cuda.synchronize()
        for r in range(2):
            with torch.cuda.stream(streams[r]):
                graphs[r].replay()
        torch.cuda.synchronize()
        assert all(c.async_error() == 0 for c in comms)
        for j, (k, c) in enumerate(seq):
            if k == "allreduce":
                want = [oracle.all_reduce(ins[j], 7, 0)] * 2
            elif k == "reducescatter":
                want = oracle.reduce_scatter(ins[j], 7, 0)
            elif k == "allgather":
                want = [oracle.all_gather(ins[j])] * 2
            else:
                want = [None, oracle.reduce(ins[j], 7, 0, 1)]
            for r in range(2):
                if want[r] is not None:
                    assert np.array_equal(ys[r][j].cpu().numpy(), want[r]), f"replay {it} op {j} ({k}) rank {r}"


REF_GRAPH_ENVS = [
    {"NCCL_AMD_REF_ORDER": "1", "NCCL_BUFFSIZE": "16384", "NCCL_MAX_CTAS": "6"},
    {"NCCL_ALGO": "RING", "NCCL_BUFFSIZE": "16384", "NCCL_MAX_CTAS": "6"},
    {"NCCL_AMD_REF_ORDER": "1", "NCCL_PROTO": "LL", "NCCL_LL_BUFFSIZE": "65536", "NCCL_MAX_CTAS": "6"},
    # reference parts shared by several workgroups (CollArgs::refSub)
    {"NCCL_AMD_REF_ORDER": "1", "NCCL_BUFFSIZE": "16384", "NCCL_AMD_REF_NCHANNELS": "6",
     "NCCL_AMD_MIN_CHANNEL_BYTES": "1024"},
]


@pytest.mark.parametrize("env", REF_GRAPH_ENVS, ids=["reforder", "ring", "reforder-ll", "reforder-sub"])
def test_hipgraph_reference_order_allreduce(built, env):
    """The reference-partition AllReduces (NCCL_AMD_REF_ORDER's direct kernel, the ring) captured in one hipGraph per
    rank — 3 ranks, bf16 (every hop rounds, so the fold order shows) at sizes spanning one and many channel parts
    and loops — and replayed with fresh inputs: the per-channel loop geometry is recomputed by every launch and the
    step counters continue across replays, bit-exact vs the reference's order every time."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    keys = ("NCCL_AMD_REF_ORDER", "NCCL_BUFFSIZE", "NCCL_MAX_CTAS", "NCCL_ALGO", "NCCL_PROTO", "NCCL_LL_BUFFSIZE",
            "NCCL_AMD_REF_NCHANNELS", "NCCL_AMD_MIN_CHANNEL_BYTES")
    saved = {k: os.environ.get(k) for k in keys}
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update(env)
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    n, counts, dt = 3, (3000, 100_003, 1 << 20), 9
    comms = []
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        comms = nccl_amd.Communicator.init_all([0] * n)
        streams = [nccl_amd.dedicated_stream(0) for _ in range(n)]
        bufs = [[(G.to_device(np.zeros(c, np.uint16), dev)[1], G.to_device(np.zeros(c, np.uint16), dev)[1])
                 for c in counts] for _ in range(n)]
        graphs = [torch.cuda.CUDAGraph() for _ in range(n)]
        torch.cuda.synchronize()
        for r in range(n):
            with torch.cuda.graph(graphs[r], stream=streams[r]):
                for c, (x, y) in zip(counts, bufs[r]):
                    comms[r].all_reduce_raw(x.data_ptr(), y.data_ptr(), c, dt, 0, streams[r].cuda_stream)
        for it in range(3):
            ins = [G.make_inputs(n, dt, c, seed=700 + 10 * it + j) for j, c in enumerate(counts)]
            for r in range(n):
                for j, (x, _) in enumerate(bufs[r]):
                    x.copy_(torch.from_numpy(ins[j][r].view(np.uint8).copy()))
            torch.cuda.synchronize()
            for r in range(n):
                with torch.cuda.stream(streams[r]):
                    graphs[r].replay()
            torch.cuda.synchronize()
            assert all(c.async_error() == 0 for c in comms)
            for j, c in enumerate(counts):
                want = G.expected("allreduce", ins[j], dt, 0)[0]
                assert not np.array_equal(want, G.oracle.all_reduce(ins[j], dt, 0)) or c == 3000, \
                    "inputs do not tell the reference order from the one-loop order"
                for r in range(n):
                    got = G.from_device(bufs[r][j][1], np.uint16)
                    assert G.same_bits(got, want, dt), f"{env} replay {it} count {c} rank {r}"
    finally:
        for cm in comms:
            if cm.ptr:
                cm.destroy()
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v


def test_init_rank_in_group_single_thread(built):
    import torch
    import nccl_amd
    torch.cuda.set_device(0)
    lib = nccl_amd.load()
    uid = nccl_amd._uid(nccl_amd.get_unique_id())
    cs = [ctypes.c_void_p(), ctypes.c_void_p()]
    assert lib.ncclGroupStart() == 0
    for r in range(2):
        assert lib.ncclCommInitRank(ctypes.byref(cs[r]), 2, uid, r) == 0
    assert lib.ncclGroupEnd() == 0
    comms = [nccl_amd.Communicator(c.value) for c in cs]
    assert [c.rank for c in comms] == [0, 1] and all(c.nranks == 2 for c in comms)
    from tests import gpu_cases as G
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    errs = G.run_case(list(zip(comms, streams)), "allreduce", 9, 0, 123_457, 0, seed=3)
    for c in comms:
        c.destroy()
    assert not errs, errs


def test_spin_timeout_reports_async_error(built):
    """Only one rank launches: its kernel must give up after NCCL_AMD_SPIN_TIMEOUT_MS and the comm
    must report ncclSystemError, then refuse further work (reference async-error semantics)."""
    import torch
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    old = os.environ.get("NCCL_AMD_SPIN_TIMEOUT_MS")
    os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "1500"
    try:
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0])
    finally:
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = old or "30000"
    x = torch.ones(1 << 20, device="cuda")
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    t0 = time.time()
    comms[0].allreduce(x, y, nccl_amd.SUM, stream=s)
    s.synchronize()
    assert time.time() - t0 < 30
    assert comms[0].async_error() == 2  # ncclSystemError
    with pytest.raises(nccl_amd.NcclError):
        comms[0].allreduce(x, y, nccl_amd.SUM, stream=s)
    comms[0].abort()
    comms[1].abort()


def test_abort_unblocks_stuck_collective(built):
    import torch
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0])
    x = torch.ones(1 << 20, device="cuda")
    y = torch.empty_like(x)
    s = torch.cuda.Stream()
    comms[0].allreduce(x, y, nccl_amd.SUM, stream=s)  # peer never joins
    time.sleep(0.5)
    t0 = time.time()
    comms[0].abort()  # sets the abort word, waits for the kernel to notice
    assert time.time() - t0 < 20
    comms[1].destroy()


@pytest.mark.parametrize("dtype,op", [(7, 0), (9, 0), (2, 3), (6, 4)])
def test_group_aggregates_small_allreduces(two_comms, dtype, op):
    """A group of many small AllReduce ops (one LL launch per run, group.cc) interleaved with a
    ReduceScatter that breaks the run; every result bit-exact vs the oracle."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    comms, streams = two_comms
    n = 2
    counts = [1, 3, 100, 4096, 777, 20_000, 8, 12_345] * 5  # 40 ops: more than one 32-op batch
    rs_count = 4096 * n
    ins = [G.make_inputs(n, dtype, cnt, seed=300 + i) for i, cnt in enumerate(counts)]
    rs_in = G.make_inputs(n, dtype, rs_count, seed=999)
    bufs = []
    for r in range(n):
        per = []
        for i, cnt in enumerate(counts):
            _, sv = G.to_device(ins[i][r], "cuda")
            _, rv = G.to_device(np.zeros(cnt, dtype=ins[i][r].dtype), "cuda")
            per.append((sv, rv))
        _, rss = G.to_device(rs_in[r], "cuda")
        _, rsr = G.to_device(np.zeros(rs_count // n, dtype=rs_in[r].dtype), "cuda")
        bufs.append((per, rss, rsr))
    torch.cuda.synchronize()
    with nccl_amd.group():
        for r in range(n):
            per, rss, rsr = bufs[r]
            s = streams[r].cuda_stream
            for i, cnt in enumerate(counts):
                if i == 20:
                    comms[r].reduce_scatter_raw(rss.data_ptr(), rsr.data_ptr(), rs_count // n, dtype, op, s)
                comms[r].all_reduce_raw(per[i][0].data_ptr(), per[i][1].data_ptr(), cnt, dtype, op, s)
    torch.cuda.synchronize()
    assert all(c.async_error() == 0 for c in comms)
    npdt = ins[0][0].dtype
    for i, cnt in enumerate(counts):
        want = G.expected("allreduce", ins[i], dtype, op)[0]
        for r in range(n):
            got = G.from_device(bufs[r][0][i][1], npdt)
            assert G.same_bits(got, want, dtype), f"op {i} (count {cnt}) rank {r}"
    want_rs = G.expected("reducescatter", rs_in, dtype, op)
    for r in range(n):
        assert G.same_bits(G.from_device(bufs[r][2], npdt), want_rs[r], dtype)


def _tuner_worker(force, nch, q):
    try:
        os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "30000"
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        plugin = os.path.join(root, "tests", "native", "libnccl-tuner-test.so")
        os.environ["NCCL_TUNER_PLUGIN"] = plugin
        os.environ["TEST_TUNER_FORCE"] = force
        os.environ["TEST_TUNER_NCH"] = str(nch)
        logf = f"/tmp/nccl_amd_tuner_{force}_{os.getpid()}.log"
        os.environ["NCCL_DEBUG"] = "TRACE"
        os.environ["NCCL_DEBUG_FILE"] = logf
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0])
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        cs = list(zip(comms, streams))
        errs = []
        for i, (coll, count) in enumerate((("allreduce", 1024), ("allreduce", 16_384), ("allreduce", 300_001),
                                           ("reducescatter", 2 * 50_000), ("allgather", 20_000), ("reduce", 77_777))):
            errs += G.run_case(cs, coll, 7, 0, count, 0, seed=700 + i, root=1)
        lib = ctypes.CDLL(plugin)
        calls, inits, last = lib.testTunerCalls(), lib.testTunerInits(), lib.testTunerLastFunc()
        for c in comms:
            c.destroy()
        log = open(logf).read() if os.path.exists(logf) else ""
        q.put((errs, calls, inits, last, log))
    except Exception as e:
        q.put(([f"exception {e!r}"], 0, 0, -1, ""))


@pytest.mark.parametrize("force,nch", [("ring_simple", 3), ("tree_simple", 0), ("ring_ll", 2), ("none", 0)])
def test_tuner_plugin(built, force, nch):
    """An external tuner plugin (reference ABI v6, tests/native/tuner_plugin.c) loaded through
    NCCL_TUNER_PLUGIN steers algorithm/protocol/channels; every result stays bit-exact. Runs in a fresh
    process: the plugin is loaded once per process, like the reference's (src/plugin/tuner.cc)."""
    import multiprocessing as mp
    import queue
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_tuner_worker, args=(force, nch, q))
    p.start()
    try:
        errs, calls, inits, last, log = q.get(timeout=240)
    except queue.Empty:
        p.kill()
        raise AssertionError("tuner worker timed out")
    p.join(timeout=60)
    assert not errs, errs
    assert inits == 2, inits          # one init per communicator
    assert calls >= 6, calls          # consulted for every collective
    assert last == 1, last            # ncclFuncReduce was the last call
    ar = [l for l in log.splitlines() if "AllReduce: " in l and ("->" in l or " LL " in l)]
    if force == "ring_simple":   # every AllReduce on the direct path with the plugin's 3 channels
        assert ar and all(" LL " not in l and "nch 3 " in l for l in ar), ar
    elif force == "ring_ll":     # LL wherever it fits (1024 and 16384 elements); 2 channels where they suffice
        assert sum(" LL count" in l for l in ar) >= 2 and any("nch 2 " in l for l in ar), ar


# Group aggregation beyond small AllReduces (group.cc, enqueue.cc batchable / launchBatch; reference
# enqueue.cc:405-440): each group is (name, dtype, [(coll, count, op, root)], the batches each comm must log).
# Counts follow gpu_cases.launch: ReduceScatter = total elements (n x recvcount), AllGather = sendcount.
# n = 2 fp32 size table: LL up to 128 KiB per AllReduce buffer / rank block, one-shot AllReduce up to 1 MiB.
BATCH_GROUPS = [
    ("mixed-size ReduceScatters", 9, [("reducescatter", 2 * c, 0, 0) for c in
                                      (100, 2000, 8192, 30_000, 100_000, 300_000, 70_000, 1_000_000)],
     [("LL", 4), ("staged", 4)]),
    ("AllGathers", 7, [("allgather", c, 0, 0) for c in (60_000, 100_000, 500_000)], [("staged", 3)]),
    ("Reduces max to root 1", 2, [("reduce", c, 2, 1) for c in (100_000, 400_000, 200_004)], [("staged", 3)]),
    ("one-shot AllReduces", 7, [("allreduce", c, 0, 0) for c in (40_000, 100_000, 250_000)], [("staged", 3)]),
    ("direct AllReduces, two operators", 7, [("allreduce", 1_000_000, 0, 0), ("allreduce", 600_000, 0, 0),
                                             ("allreduce", 1_000_000, 2, 0), ("allreduce", 700_001, 2, 0)],
     [("staged", 2), ("staged", 2)]),
    ("LL mix of collectives", 7, [("allreduce", 1000, 2, 0), ("allgather", 5000, 0, 0), ("allreduce", 3, 2, 0),
                                  ("reducescatter", 2 * 500, 2, 0), ("reduce", 100, 0, 0)], [("LL", 4)]),
]


def _batch_worker(q, rank=None, uid=None):
    """rank None: both ranks in this process (init_all on one GPU); else one rank of a 2-process comm."""
    try:
        import re
        os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "30000"
        logf = f"/tmp/nccl_amd_batch_{os.getpid()}.log"
        os.environ["NCCL_DEBUG"] = "TRACE"
        os.environ["NCCL_DEBUG_FILE"] = logf
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        n = 2
        mine = list(range(n)) if rank is None else [rank]
        comms = nccl_amd.Communicator.init_all([0, 0]) if rank is None else [nccl_amd.Communicator.init(n, rank, uid)]
        streams = [torch.cuda.Stream() for _ in mine]
        errs, logs = [], []
        for gi, (name, dt, ops, _) in enumerate(BATCH_GROUPS):
            ins = [G.make_inputs(n, dt, cnt, seed=900 + 10 * gi + i) for i, (_, cnt, _, _) in enumerate(ops)]
            bufs = [[] for _ in mine]
            for k, r in enumerate(mine):
                for i, (coll, cnt, op, root) in enumerate(ops):
                    _, sv = G.to_device(ins[i][r], "cuda")
                    _, rv = G.to_device(np.zeros(G.out_count(coll, n, cnt), dtype=ins[i][r].dtype), "cuda")
                    bufs[k].append((sv, rv))
            torch.cuda.synchronize()
            pos = os.path.getsize(logf) if os.path.exists(logf) else 0
            with nccl_amd.group():
                for k in range(len(mine)):
                    for i, (coll, cnt, op, root) in enumerate(ops):
                        G.launch(comms[k], coll, bufs[k][i][0], bufs[k][i][1], cnt, dt, op, root, streams[k].cuda_stream)
            torch.cuda.synchronize()
            errs += [f"{name}: async {c.async_error()}" for c in comms if c.async_error()]
            for i, (coll, cnt, op, root) in enumerate(ops):
                want = G.expected(coll, ins[i], dt, op, root)
                for k, r in enumerate(mine):
                    if coll == "reduce" and r != root:
                        continue
                    got = G.from_device(bufs[k][i][1], ins[i][r].dtype)
                    if not G.same_bits(got, want[0] if coll == "reduce" else want[r], dt):
                        errs.append(f"{name}: op {i} ({coll} {cnt}) rank {r} differs")
            with open(logf) as f:
                f.seek(pos)
                logs.append(re.findall(r"(LL|staged) batch: (\d+) ", f.read()))
        for c in comms:
            c.destroy()
        q.put((errs, logs))
    except Exception as e:
        q.put(([f"exception {e!r}"], []))


@pytest.mark.parametrize("procs", [1, 2])
def test_group_batches_every_collective(built, procs):
    """Consecutive ops of a group that plan onto the same kernel become ONE launch per comm: mixed-size
    ReduceScatters (an LL batch and a staged batch), AllGathers, Reduces, one-shot and direct AllReduces
    (split where the operator changes) and an LL mix of collectives. Every result bit-exact vs the oracle;
    the launch count is read from the NCCL_DEBUG=TRACE batch lines (fresh processes: logging starts once).
    procs=1: both ranks in one process (shared-GPU internal streams); procs=2: one process per rank."""
    import multiprocessing as mp
    import queue
    import nccl_amd
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    uid = nccl_amd.get_unique_id() if procs == 2 else None
    ps = [ctx.Process(target=_batch_worker, args=(q,) + ((r, uid) if procs == 2 else ())) for r in range(procs)]
    for p in ps:
        p.start()
    res = []
    try:
        for _ in ps:
            res.append(q.get(timeout=240))
    except queue.Empty:
        for p in ps:
            p.kill()
        raise AssertionError("batch worker timed out")
    for p in ps:
        p.join(timeout=60)
    for errs, _ in res:
        assert not errs, errs
    for gi, (name, _, _, want) in enumerate(BATCH_GROUPS):
        got = sorted((k, int(v)) for _, logs in res for k, v in logs[gi])
        assert got == sorted(want * 2), (name, got)  # one batch per comm (rank)


def test_nonblocking_init_from_one_thread(built):
    """config.blocking = 0 (reference init.cc, nccl.h.in:84-108): ncclCommInitRankConfig returns
    ncclInProgress at once, so ONE thread can create both ranks without a group; ncclCommGetAsyncError
    reports ncclInProgress until each is ready, then the comms work normally."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    torch.cuda.set_device(0)
    uid = nccl_amd.get_unique_id()
    cfg = nccl_amd.Config.default(blocking=0)
    comms = [nccl_amd.Communicator.init(2, r, uid, cfg) for r in range(2)]
    states = [c.async_error() for c in comms]
    assert all(s in (0, 7) for s in states), states
    for c in comms:
        c.wait_ready(120)
    assert [c.async_error() for c in comms] == [0, 0]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    errs = G.run_case(list(zip(comms, streams)), "allreduce", 7, 0, 77_777, 0, seed=11)
    for c in comms:
        c.destroy()
    assert not errs, errs


def test_nonblocking_init_reports_a_failed_mapping_check(built, monkeypatch):
    """A non-blocking init whose mapping check fails (every rank's stores dropped, NCCL_AMD_MAPCHECK_FAULT=1):
    ncclCommGetAsyncError turns from ncclInProgress to ncclSystemError on both ranks, and the handles still destroy
    cleanly (reference: a failed non-blocking init is reported through the async error, init.cc:3449)."""
    import time
    import torch
    import nccl_amd
    torch.cuda.set_device(0)
    monkeypatch.setenv("NCCL_AMD_MAPCHECK_FAULT", "1")
    uid = nccl_amd.get_unique_id()
    cfg = nccl_amd.Config.default(blocking=0)
    comms = [nccl_amd.Communicator.init(2, r, uid, cfg) for r in range(2)]
    t0 = time.time()
    while any(c.async_error() == 7 for c in comms) and time.time() - t0 < 60:
        time.sleep(0.05)
    assert [c.async_error() for c in comms] == [2, 2]
    for c in comms:
        c.destroy()


def test_communicator_churn_releases_resources(built):
    """Create, use and destroy communicators many times (2 ranks in one process, then windows too):
    device memory must return to where it started — staging, flags, counters, LL areas, IPC maps,
    internal streams and events are all released by ncclCommDestroy."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def cycle(i):
        comms = nccl_amd.Communicator.init_all([0, 0])
        errs = G.run_case(list(zip(comms, streams)), "allreduce", 7, 0, 70_001 if i % 2 else 1000, 0, seed=i)
        for c in comms:
            c.destroy()
        return errs

    assert not cycle(0)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0, _ = torch.cuda.mem_get_info()
    for i in range(1, 25):
        errs = cycle(i)
        assert not errs, errs
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free1, _ = torch.cuda.mem_get_info()
    # each communicator holds > 1 GiB of staging: a leak of even one would show
    assert free0 - free1 < (256 << 20), f"device memory not released: {(free0 - free1) >> 20} MiB lost"


def test_init_rank_scalable_and_mem_stats(built):
    """ncclCommInitRankScalable (reference init.cc:2695-2728) with three ids, two ranks created from one
    thread (non-blocking config), then an AllReduce bit-exact vs the oracle; ncclCommMemStats (reference
    mem_manager.cc:1010-1047): everything the communicator holds is persistent, > 1 GiB of staging."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    uids = [nccl_amd.get_unique_id() for _ in range(3)]
    cfg = nccl_amd.Config.default(blocking=0)
    comms = [nccl_amd.Communicator.init(2, r, uids, cfg) for r in range(2)]
    for c in comms:
        c.wait_ready(120)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    errs = G.run_case(list(zip(comms, streams)), "allreduce", 7, 0, 123_457, 0, seed=21)
    stats = [{s.name: c.mem_stats(s) for s in nccl_amd.MemStat} for c in comms]
    for c in comms:
        c.destroy()
    assert not errs, errs
    for st in stats:
        assert st["GPU_MEM_TOTAL"] == st["GPU_MEM_PERSIST"] > (1 << 30), st
        assert st["GPU_MEM_SUSPEND"] == 0 and st["GPU_MEM_SUSPENDED"] == 0, st


def test_group_simulate_end_launches_nothing(two_comms):
    """ncclGroupSimulateEnd (reference group.cc:116-123): the group's ops are planned, not launched, and the
    cost model's estimate comes back (µs in the C struct, seconds through the nccl4py mirror); the comms keep
    working afterwards (planning a simulated group changes no device-visible state)."""
    import torch
    import nccl_amd
    import oracle
    comms, streams = two_comms
    est = {}
    for count in (1024, 1 << 16, 1 << 24):
        ins = _inputs(2, count, seed=count % 97)
        sends = [torch.from_numpy(x).cuda() for x in ins]
        recvs = [torch.zeros(count, device="cuda") for _ in range(2)]
        torch.cuda.synchronize()
        nccl_amd.group_start()
        for c, s, x, y in zip(comms, streams, sends, recvs):
            c.allreduce(x, y, nccl_amd.SUM, stream=s)
        sim = nccl_amd.group_end(simulate=True)
        torch.cuda.synchronize()
        assert not recvs[0].any() and not recvs[1].any(), "a simulated group launched work"
        est[count] = sim.estimated_time
        with nccl_amd.group():
            for c, s, x, y in zip(comms, streams, sends, recvs):
                c.allreduce(x, y, nccl_amd.SUM, stream=s)
        torch.cuda.synchronize()
        want = oracle.all_reduce(ins, 7, 0)
        for y in recvs:
            assert np.array_equal(y.cpu().numpy(), want)
    assert 0 < est[1024] <= est[1 << 16] < est[1 << 24], est
    assert est[1024] < 20e-6 and est[1 << 24] > 100e-6, est  # LL latency vs 64 MiB over one xGMI link


def test_reference_buffer_and_channel_knobs(built):
    """NCCL_BUFFSIZE (reference env.rst :857: one channel's buffer towards one peer) sets the staging slot
    size, visible in ncclCommMemStats; NCCL_MAX_NCHANNELS caps the channels; results stay bit-exact."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    old = {k: os.environ.get(k) for k in ("NCCL_BUFFSIZE", "NCCL_MAX_NCHANNELS", "NCCL_MIN_NCHANNELS")}
    os.environ.update(NCCL_BUFFSIZE=str(256 << 10), NCCL_MAX_NCHANNELS="16", NCCL_MIN_NCHANNELS="4")
    try:
        comms = nccl_amd.Communicator.init_all([0, 0])
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    errs = G.run_case(list(zip(comms, streams)), "allreduce", 7, 0, 3_000_017, 0, seed=23)
    total = comms[0].mem_stats()
    for c in comms:
        c.destroy()
    assert not errs, errs
    slab = 16 * 2 * 2 * 2 * (128 << 10)  # channels x kinds x slots x ranks x (BUFFSIZE / 2 slots)
    assert slab <= total < slab + (64 << 20), (total, slab)


@pytest.mark.parametrize("count", [1_000, 300_001, 4_000_037])
def test_collectives_on_pinned_host_buffers(two_comms, count):
    """Pinned host buffers as send and receive buffers (the reference's pointer check accepts any pointer with a
    device mapping, argcheck.cc:12-28): the kernels read and write them across PCIe, on the LL and staged paths."""
    import torch
    import nccl_amd
    import oracle
    comms, streams = two_comms
    ins = _inputs(2, count, seed=31)
    sends = [torch.from_numpy(x).pin_memory() for x in ins]
    recvs = [torch.zeros(count, dtype=torch.float32).pin_memory() for _ in range(2)]
    gathered = [torch.zeros(2 * count, dtype=torch.float32).pin_memory() for _ in range(2)]
    torch.cuda.synchronize()
    nccl_amd.group_start()
    for c, s, x, y in zip(comms, streams, sends, recvs):
        c.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, s.cuda_stream)
    nccl_amd.group_end()
    torch.cuda.synchronize()
    want = oracle.all_reduce(ins, 7, 0)
    for r, y in enumerate(recvs):
        got = y.numpy()
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"AllReduce rank {r}: {bad.size} mismatches, first {bad[:6].tolist()}"
    nccl_amd.group_start()
    for c, s, x, y in zip(comms, streams, sends, gathered):
        c.all_gather_raw(x.data_ptr(), y.data_ptr(), count, 7, s.cuda_stream)
    nccl_amd.group_end()
    torch.cuda.synchronize()
    for r, y in enumerate(gathered):
        assert np.array_equal(y.numpy(), np.concatenate(ins)), f"AllGather rank {r}"
    # ReduceScatter of the gathered (2 * count) buffers, and Reduce to root 1, host buffers on both sides
    scat = [torch.zeros(count, dtype=torch.float32).pin_memory() for _ in range(2)]
    nccl_amd.group_start()
    for c, s, x, y in zip(comms, streams, gathered, scat):
        c.reduce_scatter_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, s.cuda_stream)
    nccl_amd.group_end()
    torch.cuda.synchronize()
    want_rs = oracle.reduce_scatter([y.numpy().copy() for y in gathered], 7, 0)
    for r, y in enumerate(scat):
        assert np.array_equal(y.numpy(), want_rs[r]), f"ReduceScatter rank {r}"
    red = torch.zeros(count, dtype=torch.float32).pin_memory()
    nccl_amd.group_start()
    for r, (c, s, x) in enumerate(zip(comms, streams, sends)):
        c.reduce_raw(x.data_ptr(), red.data_ptr() if r == 1 else None, count, 7, 0, 1, s.cuda_stream)
    nccl_amd.group_end()
    torch.cuda.synchronize()
    assert np.array_equal(red.numpy(), oracle.reduce(ins, 7, 0, 1)), "Reduce"
    assert all(c.async_error() == 0 for c in comms)


@pytest.mark.parametrize("count", [(1 << 18) + 3, 3 << 20])
def test_one_rank_copy_on_pinned_host_buffers(built, count):
    """The one-rank path with a pinned host buffer on either side (the copy's grid is capped for PCIe at >= 1 MiB,
    NCCL_AMD_HOST_COPY_GRID): host -> host, host -> device, device -> host, bit-exact."""
    import torch
    import nccl_amd
    torch.cuda.set_device(0)
    comm = nccl_amd.Communicator.init_all([0])[0]
    try:
        x = torch.randn(count).pin_memory()
        st = torch.cuda.current_stream().cuda_stream
        for src_dev, dst_dev in ((False, False), (False, True), (True, False)):
            src = x.cuda() if src_dev else x
            dst = torch.zeros(count, device="cuda") if dst_dev else torch.zeros(count).pin_memory()
            torch.cuda.synchronize()
            comm.all_reduce_raw(src.data_ptr(), dst.data_ptr(), count, 7, 0, st)
            torch.cuda.synchronize()
            assert torch.equal(dst.cpu(), x), (src_dev, dst_dev)
    finally:
        comm.destroy()
