"""GPU parity tests: the HIP kernels behind the C ABI vs the CPU oracle (bit-exact for every type,
including floats, because the kernels fold in the oracle's order with the same per-hop rounding).

Multi-rank cases run several ranks on the ONE GPU of the test box: single-process (ncclCommInitAll
with a repeated device, NCCL_MULTI_RANK_GPU_ENABLE=1, reference init.cc:68) and multi-process
(ncclCommInitRank over the TCP bootstrap + HIP IPC). The 8-GPU xGMI path runs the same kernels."""
import multiprocessing as mp
import os

import numpy as np

import pytest

os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "30000")

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU test on a box without a GPU"
    return torch


def test_one_rank_all_cases(built):
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    torch.cuda.set_device(0)
    comm = nccl_amd.Communicator.init_all([0])[0]
    s = torch.cuda.Stream()
    errs = []
    for i, (coll, dt, op, count, mis) in enumerate(G.case_list(1)):
        errs += G.run_case([(comm, s)], coll, dt, op, count, mis, seed=i)
        errs += G.run_case([(comm, s)], coll, dt, op, count, mis, seed=i, inplace=True) if mis == 0 and i % 3 == 0 else []
    comm.destroy()
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("variant,grid", [("0", None), ("10", None), ("0", "13"), ("0", "3")])
def test_one_rank_copy_tile_mappings(built, monkeypatch, variant, grid):
    """The n = 1 copy (onerank.cu:49-110's cudaMemcpyAsync, here copyKernel) under the XCD-contiguous tile mapping
    (default) and the identity mapping (variant 10): byte-identical output at grids that are / are not multiples of 8,
    below 8 tiles, partial last tiles and byte tails, and with a capped grid (NCCL_AMD_COPY_GRID) striding over the
    permuted tiles."""
    torch = _torch()
    import nccl_amd
    torch.cuda.set_device(0)
    monkeypatch.setenv("NCCL_AMD_COPY_VARIANT", variant)
    if grid:
        monkeypatch.setenv("NCCL_AMD_COPY_GRID", grid)
    comm = nccl_amd.Communicator.init_all([0])[0]
    g = torch.Generator(device="cuda").manual_seed(7)
    tile = 8192
    for nbytes in (tile * 40, tile * 43, tile * 43 + 48, tile * 43 + 48 + 7, tile * 7, tile * 8 * 33 + 16, 5):
        src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda", generator=g)
        dst = torch.zeros_like(src)
        comm.allreduce(src, dst, nccl_amd.SUM)
        torch.cuda.synchronize()
        assert torch.equal(src, dst), (variant, grid, nbytes)
    comm.destroy()


@pytest.mark.parametrize("nranks", [2, 3])
def test_single_process_multirank(built, nranks):
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0] * nranks)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    cs = list(zip(comms, streams))
    errs = []
    for i, (coll, dt, op, count, mis) in enumerate(G.case_list(nranks, quick=(nranks > 2))):
        for root in ([0] if coll != "reduce" else [0, nranks - 1]):
            errs += G.run_case(cs, coll, dt, op, count, mis, seed=i, root=root)
        if i % 4 == 0 and mis == 0:
            errs += G.run_case(cs, coll, dt, op, count, mis, seed=i, inplace=True)
        if errs:
            break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


def _mp_worker(rank, nranks, uid, quick, q, env=None):
    try:
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "30000"
        os.environ.update(env or {})
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        s = torch.cuda.Stream()
        errs = []
        for i, (coll, dt, op, count, mis) in enumerate(G.case_list(nranks, quick=quick)):
            root = i % nranks
            errs += G.run_case([(comm, s)], coll, dt, op, count, mis, seed=i, root=root,
                               algo=(env or {}).get("NCCL_ALGO", ""))
            if errs:
                break
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


# (nranks, env): the second group forces tiny staging slots so every channel runs many pipeline
# steps with slot reuse (credit protocol, A(s+1)-before-C(s) ordering) at test sizes.
MP_CASES = [(2, {}), (4, {}), (8, {}),
            (2, {"NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "2"}),
            (3, {"NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "1"}),
            (4, {"NCCL_AMD_SLOT_BYTES": "8192", "NCCL_AMD_NSLOTS": "3", "NCCL_MAX_CTAS": "7"}),
            (3, {"NCCL_ALGO": "ONESHOT", "NCCL_AMD_SLOT_BYTES": "16384"}),
            (3, {"NCCL_PROTO": "LL"}),
            (2, {"NCCL_PROTO": "^LL"}),
            (2, {"NCCL_ALGO": "DIRECT"}),
            (3, {"NCCL_AMD_AG_PULL": "1", "NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "2"}),
            (4, {"NCCL_AMD_AG_PULL": "1"}),
            # the push gather (the default before round 5; NCCL_AMD_AG_PULL=0 keeps it)
            (4, {"NCCL_AMD_AG_PULL": "0"}),
            (3, {"NCCL_AMD_AG_PULL": "0", "NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "2"}),
            (3, {"NCCL_AMD_RS_PULL": "1", "NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "1"}),
            (4, {"NCCL_AMD_RS_PULL": "1", "NCCL_AMD_AG_PULL": "1"}),
            (4, {"NCCL_ALGO": "RING"}), (3, {"NCCL_ALGO": "TREE", "NCCL_AMD_SLOT_BYTES": "4096"}),
            # the reference's ring partition with many channel parts and loops at test sizes (small chunks): the
            # ring itself, and the direct kernel walking the same partition (NCCL_AMD_REF_ORDER)
            (3, {"NCCL_ALGO": "RING", "NCCL_BUFFSIZE": "16384", "NCCL_MAX_CTAS": "5"}),
            (3, {"NCCL_AMD_REF_ORDER": "1", "NCCL_BUFFSIZE": "16384", "NCCL_MAX_CTAS": "5"}),
            # ... with each reference part shared by several workgroups (CollArgs::refSub; 1 KiB sub-chunks so the
            # 8 KiB chunks split too): sub-chunk edges, ragged last loops, empty sub-chunks
            (3, {"NCCL_ALGO": "RING", "NCCL_BUFFSIZE": "16384", "NCCL_AMD_REF_NCHANNELS": "5",
                 "NCCL_AMD_MIN_CHANNEL_BYTES": "1024"}),
            (3, {"NCCL_AMD_REF_ORDER": "1", "NCCL_BUFFSIZE": "16384", "NCCL_AMD_REF_NCHANNELS": "5",
                 "NCCL_AMD_MIN_CHANNEL_BYTES": "1024"}),
            (4, {"NCCL_AMD_REF_ORDER": "1", "NCCL_PROTO": "LL", "NCCL_LL_BUFFSIZE": "65536",
                 "NCCL_AMD_REF_NCHANNELS": "3", "NCCL_AMD_MIN_CHANNEL_BYTES": "512"}),
            (4, {"NCCL_AMD_REF_ORDER": "1", "NCCL_AMD_SLOT_BYTES": "4096"}),
            # ... on the reference's RING/LL and RING/LL128 partitions (small protocol buffers: many parts and loops)
            (3, {"NCCL_AMD_REF_ORDER": "1", "NCCL_PROTO": "LL", "NCCL_LL_BUFFSIZE": "65536", "NCCL_MAX_CTAS": "6"}),
            (2, {"NCCL_AMD_REF_ORDER": "1", "NCCL_PROTO": "LL128", "NCCL_LL128_BUFFSIZE": "131072"}),
            (3, {"NCCL_ALGO": "RING", "NCCL_PROTO": "LL", "NCCL_LL_BUFFSIZE": "65536", "NCCL_MAX_CTAS": "4"}),
            # cross-process memory: every dma-buf import refused -> the hipIpc handle fallback (ipc.cc); legacy
            # handles only (NCCL_AMD_IPC=legacy) run where the runtime is 7.2+, see test_legacy_ipc_runtime_gate
            (3, {"NCCL_AMD_IPC_FAIL_DMABUF": "1"}),
            # the LL128-class protocol (LL64 lines): forced for everything it fits, and in its size-table range
            (3, {"NCCL_PROTO": "LL128"}), (4, {"NCCL_AMD_LL128": "1"})]


def _mp_id(n, env):
    return f"n{n}-" + ("-".join(f"{k.replace('NCCL_AMD_', '').replace('NCCL_', '')}={v}" for k, v in env.items())
                       or "default")


@pytest.mark.parametrize("nranks,env", MP_CASES, ids=[_mp_id(n, e) for n, e in MP_CASES])
def test_multi_process(built, nranks, env):
    _torch()
    import nccl_amd
    uid = nccl_amd.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mp_worker, args=(r, nranks, uid, nranks > 2 or bool(env), q, env)) for r in range(nranks)]
    for p in ps:
        p.start()
    import queue
    import time
    results = {}
    t0 = time.time()
    while len(results) < nranks and time.time() - t0 < 900:
        try:
            r, errs = q.get(timeout=30)
            results[r] = errs
        except queue.Empty:
            alive = sum(p.is_alive() for p in ps)
            print(f"[multi_process n={nranks}] waiting: {len(results)} done, {alive} alive, {time.time() - t0:.0f}s",
                  flush=True)
            if alive == 0:
                break
    for p in ps:
        if p.is_alive() and len(results) < nranks:
            p.kill()
    assert len(results) == nranks, f"only {len(results)} of {nranks} ranks reported"
    for p in ps:
        p.join(timeout=60)
    bad = [e for r in sorted(results) for e in results[r]]
    assert not bad, "\n".join(bad[:20])


def _torch_hip_runtime():
    import torch
    parts = (torch.version.hip or "0.0").split(".")
    return int(parts[0]) * 100 + int(parts[1])


def test_legacy_ipc_runtime_gate(built):
    """NCCL_AMD_IPC=legacy (hipIpc handles) is refused on HIP runtimes older than 7.2 — the
    one bound in a torch process is torch's bundled runtime, whose hipIpcOpenMemHandle stalls at 2 GiB — with a
    clean ncclSystemError naming that runtime, within seconds, never a hang; on a 7.2+ runtime it runs and is
    bit-exact."""
    import queue
    import time
    _torch()
    import nccl_amd
    old = _torch_hip_runtime() < 702
    uid = nccl_amd.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    env = {"NCCL_AMD_IPC": "legacy"}
    ps = [ctx.Process(target=_mp_worker, args=(r, 2, uid, True, q, env)) for r in range(2)]
    t0 = time.time()
    for p in ps:
        p.start()
    results = {}
    while len(results) < 2 and time.time() - t0 < 300:
        try:
            r, errs = q.get(timeout=30)
            results[r] = errs
        except queue.Empty:
            if not any(p.is_alive() for p in ps):
                break
    for p in ps:
        if p.is_alive():
            p.kill()
        p.join(timeout=60)
    assert len(results) == 2, f"only {len(results)} of 2 ranks reported"
    errs = [e for r in sorted(results) for e in results[r]]
    if old:
        assert len(errs) == 2 and all("refused on HIP runtime" in e and "libamdhip64" in e for e in errs), errs
        assert time.time() - t0 < 200
    else:
        assert not errs, errs


def test_reference_example_known_answer(built):
    """docs/examples/03_collectives/01_allreduce/c/main.cc:99-168: 32 Mi floats per rank, sendbuff[i][0] = i
    and zeros elsewhere, group of per-rank ncclAllReduce; element 0 must be n(n-1)/2 exactly (and the
    rest zero) — here with 3 ranks on the one GPU, at the example's full size."""
    torch = _torch()
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    n, size = 3, 32 * 1024 * 1024
    comms = nccl_amd.Communicator.init_all([0] * n)
    streams = [torch.cuda.Stream() for _ in range(n)]
    sends = [torch.zeros(size, device="cuda") for _ in range(n)]
    recvs = [torch.full((size,), -1.0, device="cuda") for _ in range(n)]
    for i in range(n):
        sends[i][0] = i
    torch.cuda.synchronize()
    with nccl_amd.group():
        for c, s, x, y in zip(comms, streams, sends, recvs):
            c.allreduce(x, y, nccl_amd.SUM, stream=s)
    torch.cuda.synchronize()
    for y in recvs:
        assert float(y[0]) == n * (n - 1) / 2
        assert int(torch.count_nonzero(y[1:])) == 0
    for c in comms:
        c.destroy()


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_tolerance_vs_fp32_reference(built, dtype):
    """contrib/nccl_ubx/tests/distributed/_workers/_run_ubx_op.py:65-128 convention: randn inputs
    (seed 42+rank), reference = fp32 sum, bf16 atol 0.0625 / rtol 0.02, fp32 atol 1e-4 / rtol 1e-3."""
    torch = _torch()
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    n, count = 4, 1 << 20
    comms = nccl_amd.Communicator.init_all([0] * n)
    streams = [torch.cuda.Stream() for _ in range(n)]
    dt = getattr(torch, dtype)
    xs = []
    for r in range(n):
        g = torch.Generator(device="cuda")
        g.manual_seed(42 + r)
        xs.append(torch.randn(count, device="cuda", generator=g).to(dt))
    ys = [torch.empty_like(x) for x in xs]
    torch.cuda.synchronize()
    with nccl_amd.group():
        for c, s, x, y in zip(comms, streams, xs, ys):
            c.allreduce(x, y, nccl_amd.SUM, stream=s)
    torch.cuda.synchronize()
    ref = sum(x.float() for x in xs)
    atol, rtol = (0.0625, 0.02) if dtype == "bfloat16" else (1e-4, 1e-3)
    for y in ys:
        torch.testing.assert_close(y.float(), ref, atol=atol, rtol=rtol)
    for c in comms:
        c.destroy()


def test_ll_epoch_wraparound(built):
    """LL flags are 32-bit epochs with parity double-buffering; start just below 2^32 (reference
    TEST_LL_CLEANUP idea) and run many LL AllReduces across the wrap, checking each bit-exactly."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    os.environ["NCCL_AMD_LL_EPOCH_BASE"] = str(2**32 - 5)
    try:
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0])
    finally:
        os.environ.pop("NCCL_AMD_LL_EPOCH_BASE")
    streams = [torch.cuda.Stream() for _ in range(2)]
    cs = list(zip(comms, streams))
    errs = []
    for i in range(12):
        errs += G.run_case(cs, "allreduce", 7 if i % 2 else 9, 0, 1000 + 37 * i, 0, seed=500 + i)
    for c in comms:
        c.destroy()
    assert not errs, errs


@pytest.mark.parametrize("nranks", [2, 3])
def test_ll_reducescatter_allgather(built, nranks):
    """LL protocol for the blocked collectives (8-byte aligned rank blocks within the LL range): every
    type and op, ragged payload tails (blocks of 8k+2 / 8k+4 bytes are excluded by the alignment rule,
    so the tails are whole 8-byte payloads across channel parts), in place and out of place."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0] * nranks)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    cs = list(zip(comms, streams))
    errs = []
    i = 0
    for dtype in (7, 9, 6, 2, 3, 4, 0, 1, 5, 8, 10, 11):
        es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
        for block_bytes in (8, 1024, 24_008):
            block = max(1, block_bytes // es)
            for coll, ops in (("reducescatter", (0, 1, 2, 3, 4)), ("allgather", (0,))):
                for op in ops:
                    count = block * nranks if coll == "reducescatter" else block
                    errs += G.run_case(cs, coll, dtype, op, count, 0, seed=900 + i)
                    if op == 0:
                        errs += G.run_case(cs, coll, dtype, op, count, 0, seed=901 + i, inplace=True)
                    i += 1
        if errs:
            break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("nranks", [2, 3])
def test_ll128_every_collective(built, nranks, monkeypatch):
    """The LL128-class protocol (kernels.h ll64ChannelOp, NCCL_PROTO=LL128): 64-byte lines of 56 payload bytes.
    Every collective, type and op, sizes that end mid-line, mid-payload and on channel-part boundaries,
    in place, unaligned bases; bit-exact vs the oracle (same fold order as every other path)."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    monkeypatch.setenv("NCCL_PROTO", "LL128")
    monkeypatch.setenv("NCCL_AMD_LL128_CHANNEL_BYTES", "4096")  # many channels even at small sizes
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0] * nranks)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    cs = list(zip(comms, streams))
    errs = []
    i = 0
    for dtype in (7, 9, 6, 2, 3, 4, 0, 1, 5, 8, 10, 11):
        es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
        for nbytes in (8, 56, 64, 1000, 4096 * 3 + 56 * 5, 100_000):
            count = max(1, nbytes // es)
            ops = (0, 1, 2, 3, 4) if nbytes in (1000, 100_000) else (0,)
            for op in ops:
                errs += G.run_case(cs, "allreduce", dtype, op, count + (i % 3), 0, seed=1200 + i)
                errs += G.run_case(cs, "reduce", dtype, op, count, 0, seed=1300 + i, root=i % nranks)
                blk = max(1, (nbytes // 8) * 8 // es)  # blocked collectives: 8-byte multiple rank blocks
                errs += G.run_case(cs, "reducescatter", dtype, op, blk * nranks, 0, seed=1400 + i)
                i += 1
            errs += G.run_case(cs, "allgather", dtype, 0, max(1, (nbytes // 8) * 8 // es), 0, seed=1500 + i)
            errs += G.run_case(cs, "allreduce", dtype, 0, count, 0, seed=1600 + i, inplace=True)
            errs += G.run_case(cs, "allreduce", dtype, 0, count, 1, seed=1700 + i)  # misaligned bases
        if errs:
            break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


def test_ll_and_ll128_share_channels(built, monkeypatch):
    """LL and LL64 ops interleaved on the same channels (shared epochs, separate line areas): sizes alternating
    between the LL range and the LL128 range, one op at a time and in group batches, across the 32-bit epoch
    wrap; every result bit-exact."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    monkeypatch.setenv("NCCL_AMD_LL128", "1")
    monkeypatch.setenv("NCCL_AMD_LL_EPOCH_BASE", str(2**32 - 7))
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0, 0])
    streams = [torch.cuda.Stream() for _ in range(3)]
    cs = list(zip(comms, streams))
    errs = []
    for i in range(16):
        count = 1000 + 13 * i if i % 2 else 60_000 + 101 * i  # 4 KB (LL) / 240 KB (LL128 at n=3)
        errs += G.run_case(cs, "allreduce", 7, 0, count, 0, seed=2000 + i)
    # group batches: several LL128 ops in one launch, then an LL batch
    for k in range(3):
        errs += G.run_group(cs, [("allreduce", 9, 0, 50_000 + 7 * j) for j in range(5)], seed=2100 + k)
        errs += G.run_group(cs, [("allreduce", 7, 2, 300 + j) for j in range(6)], seed=2200 + k)
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


def test_counts_above_int32(built):
    """Maximum-size edge: element counts past 2^31 (uint8, so 2 GiB+ buffers) through the one-rank copy and
    the two-rank staged AllReduce, ReduceScatter and AllGather, checked elementwise on the device against
    the modular sums of two closed-form inputs (size-independent property: (a + b) mod 256)."""
    torch = _torch()
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    big = (1 << 31) + 4099
    idx = torch.arange(big, device="cuda", dtype=torch.int64)
    xs = [(idx % 251).to(torch.uint8), ((idx * 7 + 3) % 253).to(torch.uint8)]
    want = ((xs[0].to(torch.int16) + xs[1].to(torch.int16)) % 256).to(torch.uint8)
    del idx
    # one rank: the copy kernel
    c1 = nccl_amd.Communicator.init_all([0])[0]
    y = torch.empty_like(xs[0])
    s = torch.cuda.Stream()
    c1.all_reduce_raw(xs[0].data_ptr(), y.data_ptr(), big, 1, 0, s.cuda_stream)
    s.synchronize()
    assert c1.async_error() == 0 and torch.equal(y, xs[0])
    c1.destroy()
    del y
    comms = nccl_amd.Communicator.init_all([0, 0])
    streams = [torch.cuda.Stream() for _ in range(2)]
    # AllReduce
    ys = [torch.empty_like(x) for x in xs]
    with nccl_amd.group():
        for c, st, x, yy in zip(comms, streams, xs, ys):
            c.all_reduce_raw(x.data_ptr(), yy.data_ptr(), big, 1, 0, st.cuda_stream)
    torch.cuda.synchronize()
    for c, yy in zip(comms, ys):
        assert c.async_error() == 0 and torch.equal(yy, want)
    del ys
    # ReduceScatter: recvcount = big // 2 per rank (input big - big % 2 elements)
    rc = big // 2
    outs = [torch.empty(rc, dtype=torch.uint8, device="cuda") for _ in range(2)]
    with nccl_amd.group():
        for c, st, x, o in zip(comms, streams, xs, outs):
            c.reduce_scatter_raw(x.data_ptr(), o.data_ptr(), rc, 1, 0, st.cuda_stream)
    torch.cuda.synchronize()
    for r, o in enumerate(outs):
        assert comms[r].async_error() == 0 and torch.equal(o, want[r * rc:(r + 1) * rc])
    del outs
    # AllGather: sendcount = big // 2 + 1 per rank, output past 2^31
    sc = big // 2 + 1
    full = [torch.empty(2 * sc, dtype=torch.uint8, device="cuda") for _ in range(2)]
    with nccl_amd.group():
        for c, st, x, f in zip(comms, streams, xs, full):
            c.all_gather_raw(x.data_ptr(), f.data_ptr(), sc, 1, st.cuda_stream)
    torch.cuda.synchronize()
    for r, f in enumerate(full):
        assert comms[r].async_error() == 0
        assert torch.equal(f[:sc], xs[0][:sc]) and torch.equal(f[sc:], xs[1][:sc])
    for c in comms:
        c.destroy()


def test_one_byte_types_full_channel_plans(built):
    """1-byte types at sizes that plan the full 256 channels, 2 ranks in one process: every channel of
    both ranks must be resident at once (kernel register budget, tests/test_occupancy.py) — before that
    budget the uint8 / fp8 kernels fit one workgroup per CU and these cases waited forever."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0])
    streams = [torch.cuda.Stream() for _ in range(2)]
    cs = list(zip(comms, streams))
    errs = []
    for i, (coll, dt, op) in enumerate([("allreduce", 1, 0), ("allreduce", 0, 3), ("allreduce", 10, 0),
                                        ("allreduce", 11, 2), ("reducescatter", 1, 0), ("reduce", 10, 0)]):
        errs += G.run_case(cs, coll, dt, op, (64 << 20) + 6, 0, seed=700 + i)
        if errs:
            break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


# special values per dtype, in storage bits: NaNs (both signs), infinities, signed zeros, the smallest and a
# large subnormal, the largest finite values (fp8 e4m3 has no infinity)
SPECIALS = {
    7: np.array([np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, -1.1754942e-38, 3.4028235e38, -3.4028235e38,
                 1.0], dtype=np.float32),
    8: np.array([np.nan, -np.nan, np.inf, -np.inf, 0.0, -0.0, 5e-324, -2.2250738585072e-308, 1.7976931348623157e308,
                 -1.7976931348623157e308, 1.0], dtype=np.float64),
    6: np.array([0x7E00, 0xFE00, 0x7C00, 0xFC00, 0, 0x8000, 0x0001, 0x83FF, 0x7BFF, 0xFBFF, 0x3C00], dtype=np.uint16),
    9: np.array([0x7FC0, 0xFFC0, 0x7F80, 0xFF80, 0, 0x8000, 0x0001, 0x807F, 0x7F7F, 0xFF7F, 0x3F80], dtype=np.uint16),
    10: np.array([0x7F, 0xFF, 0x00, 0x80, 0x01, 0x87, 0x7E, 0xFE, 0x38], dtype=np.uint8),
    11: np.array([0x7C, 0xFC, 0x7E, 0xFE, 0x00, 0x80, 0x01, 0x83, 0x7B, 0xFB, 0x3C], dtype=np.uint8),
}


def _with_specials(inputs, dtype):
    sp = SPECIALS[dtype]
    L = len(sp)
    out = []
    for r, x in enumerate(inputs):
        y = x.copy()
        raw = y.view(sp.dtype) if sp.dtype.kind in "ui" else y
        for off, shift in ((0, 3), (1, 1), (2, 7)):  # different pairings of specials across the ranks
            idx = np.arange(off, y.size, 37)
            raw[idx] = sp[(np.arange(idx.size) + r * shift) % L]
        out.append(y)
    return out


def _int_view(dtype):
    """The integer type of dtype's width: raw element bits on the host and in torch."""
    from tests import gpu_cases as G
    return {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize]


def _comparable(ins, dtype, op):
    """Elements whose result bits are defined for Sum / Prod / Avg: at most one NaN arises in the fold (one NaN input
    and no NaN made from Inf - Inf / 0 x Inf, or none at all). Where two NaNs meet, which one an add or multiply returns
    depends on its operand order, which the compiler may commute (IEEE leaves the payload open). Min / Max (explicit
    selects) and integer types: every element."""
    from tests import gpu_cases as G
    count = ins[0].size
    if op in (2, 3) or dtype not in G.FLOAT_TYPES:
        return np.ones(count, dtype=bool)
    f = np.stack([G.oracle.to_f32(dtype, x) for x in ins])
    made = (np.isinf(f).any(0) & (f == 0).any(0)) if op == 1 else ((f == np.inf).any(0) & (f == -np.inf).any(0))
    return np.isnan(f).sum(0) + made <= 1


@pytest.mark.parametrize("dtype", [7, 8, 6, 9, 10, 11])
def test_special_float_values(built, dtype):
    """NaN / ±Inf / ±0 / subnormal / max-finite inputs, combined across 3 ranks, through every path (LL,
    one-shot, direct) and operator: bit-exact vs the oracle (any NaN matches any NaN). Subnormals must
    survive (no flush to zero, reference common.mk:103), min/max must ignore NaN like fminf/fmaxf."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0, 0])
    streams = [torch.cuda.Stream() for _ in range(3)]
    cs = list(zip(comms, streams))
    errs = []
    es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
    for count in (4096 // es * 3 + 3, 600_000 // es, 4_000_000 // es):   # LL, one-shot, direct at n = 3
        for op in (0, 1, 2, 3, 4):
            ins = _with_specials(G.make_inputs(3, dtype, count, seed=11 + op), dtype)
            errs += G.run_case(cs, "allreduce", dtype, op, count, 0, seed=0, inputs=ins)
        ins = _with_specials(G.make_inputs(3, dtype, count - count % 3, seed=5), dtype)
        errs += G.run_case(cs, "reducescatter", dtype, 0, count - count % 3, 0, seed=0, inputs=ins)
        if errs:
            break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


def _single_nan_errors(comms, streams, dtype, count, op, seed, algo=""):
    """AllReduce of special-value inputs on comms (3 ranks in this process); the elements where exactly one NaN arises
    in the fold must equal the oracle's bits (algo: the oracle's fold order, as gpu_cases.expected)."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    vt = _int_view(dtype)
    ins = _with_specials(G.make_inputs(3, dtype, count, seed=seed), dtype)
    want = G._raw(G.expected("allreduce", ins, dtype, op, 0, algo)[0])
    bufs = [torch.from_numpy(np.ascontiguousarray(x).view(vt).copy()).cuda() for x in ins]
    outs = [torch.empty_like(b) for b in bufs]
    with nccl_amd.group():
        for r, (c, st) in enumerate(zip(comms, streams)):
            c.all_reduce_raw(bufs[r].data_ptr(), outs[r].data_ptr(), count, dtype, op, st.cuda_stream)
    torch.cuda.synchronize()
    one = _comparable(ins, dtype, op) & (np.isnan(np.stack([G.oracle.to_f32(dtype, x) for x in ins])).sum(0) == 1)
    assert one.sum() > 0
    errs = []
    for r in range(3):
        got = outs[r].cpu().numpy().view(want.dtype)
        bad = np.nonzero(got[one] != want[one])[0]
        if bad.size:
            errs.append(f"dtype {dtype} op {op} count {count} rank {r}: {bad.size} of {one.sum()} single-NaN elements "
                        f"differ, e.g. {hex(int(got[one][bad[0]]))} vs {hex(int(want[one][bad[0]]))}")
    return errs


def test_single_nan_payloads(built):
    """Where exactly one rank contributes a NaN (the others finite or infinite), Sum / Prod / Avg return that NaN
    quieted, sign and payload kept, on every path (LL, one-shot, direct) — bit for bit the oracle's result — for every
    float type; fp8 NaN is sign | 0x7f on every path (round 4: the packed e5m2 encode gave 0x7e / 0xfe). Elements
    where a NaN is also produced from non-NaN inputs (Inf - Inf, 0 x Inf) are excluded: the default NaN and what
    happens when two NaNs meet are the hardware's."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0, 0])
    streams = [torch.cuda.Stream() for _ in range(3)]
    errs = []
    for dtype in (7, 8, 6, 9, 10, 11):
        es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
        for count in (4096 // es * 3 + 3, 600_000 // es, 4_000_000 // es):  # LL, one-shot, direct at n = 3
            for op in (0, 1, 4):
                errs += _single_nan_errors(comms, streams, dtype, count, op, 11 + op)
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("dtype", [7, 8, 6, 9, 10, 11])
def test_every_path_same_bits_with_specials(built, monkeypatch, dtype):
    """The paths that fold in the same order (LL, LL128 class, one-shot, direct, direct with pulls, the zero-copy kernel
    on registered buffers) must store the same bits for the same inputs — NaN sign and payload included, generated
    NaNs too, since they run on the same hardware — for every operator, except where two NaNs meet in an add or a
    multiply (below). The oracle comparison ignores NaN bits; this one does not (the round-4 e5m2 NaN encode differed
    between the LL and the packed paths)."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    monkeypatch.setenv("NCCL_MULTI_RANK_GPU_ENABLE", "1")
    torch.cuda.set_device(0)
    es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
    vt = _int_view(dtype)
    count = 48 * 1024 // es + 3
    paths = {"LL": {"NCCL_PROTO": "LL"}, "LL128": {"NCCL_PROTO": "LL128"}, "ONESHOT": {"NCCL_ALGO": "ONESHOT"},
             "DIRECT": {"NCCL_ALGO": "DIRECT", "NCCL_PROTO": "Simple"},
             "DIRECT_PULLS": {"NCCL_ALGO": "DIRECT", "NCCL_PROTO": "Simple", "NCCL_AMD_AG_PULL": "1",
                              "NCCL_AMD_RS_PULL": "1"},
             "DIRECT_PUSH": {"NCCL_ALGO": "DIRECT", "NCCL_PROTO": "Simple", "NCCL_AMD_AG_PULL": "0"},
             "REGISTERED": {"NCCL_PROTO": "Simple"}}
    results = {}
    for name, env in paths.items():
        for k in ("NCCL_PROTO", "NCCL_ALGO", "NCCL_AMD_AG_PULL", "NCCL_AMD_RS_PULL"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        comms = nccl_amd.Communicator.init_all([0, 0, 0])
        streams = [torch.cuda.Stream() for _ in range(3)]
        out = {}
        for op in (0, 1, 2, 3, 4):
            ins = _with_specials(G.make_inputs(3, dtype, count, seed=21 + op), dtype)
            bufs = [torch.from_numpy(np.ascontiguousarray(x).view(vt).copy()).cuda() for x in ins]
            outs = [torch.empty_like(b) for b in bufs]
            hs = ([c.register_buffer(b.data_ptr(), b.numel() * es) for c, b in zip(comms, bufs)] +
                  [c.register_buffer(o.data_ptr(), o.numel() * es) for c, o in zip(comms, outs)]
                  if name == "REGISTERED" else [])
            torch.cuda.synchronize()
            with nccl_amd.group():
                for r, (c, st) in enumerate(zip(comms, streams)):
                    c.all_reduce_raw(bufs[r].data_ptr(), outs[r].data_ptr(), count, dtype, op, st.cuda_stream)
            torch.cuda.synchronize()
            out[op] = [o.cpu().numpy() for o in outs]
            for i, h in enumerate(hs):
                comms[i % 3].deregister_buffer(h)
        for c in comms:
            c.destroy()
        results[name] = out
    keep = {op: _comparable(_with_specials(G.make_inputs(3, dtype, count, seed=21 + op), dtype), dtype, op)
            for op in (0, 1, 2, 3, 4)}
    errs = []
    for name, out in results.items():
        for op in out:
            for r in range(3):
                a, b = results["LL"][op][r][keep[op]], out[op][r][keep[op]]
                if not np.array_equal(a, b):
                    bad = np.nonzero(a != b)[0]
                    errs.append(f"{name} vs LL, op {op}, rank {r}: {bad.size} elements differ, first at {bad[0]}: "
                                f"{hex(int(b[bad[0]]))} vs {hex(int(a[bad[0]]))}")
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("coll", ["reducescatter", "reduce"])
@pytest.mark.parametrize("dtype", [7, 9, 10, 11])
def test_reduce_paths_same_bits_with_specials(built, monkeypatch, coll, dtype):
    """As test_every_path_same_bits_with_specials, for ReduceScatter (LL, LL128 class, direct, pulls, registered
    zero-copy) and Reduce (LL, direct; root 1): identical bits on every path, NaN included, outside the elements where
    two NaNs meet in an add or multiply."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    monkeypatch.setenv("NCCL_MULTI_RANK_GPU_ENABLE", "1")
    torch.cuda.set_device(0)
    es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
    vt = _int_view(dtype)
    per = 16 * 1024 // es + 8          # ReduceScatter: elements per rank block (16-byte aligned blocks)
    count = 3 * per if coll == "reducescatter" else 48 * 1024 // es + 3
    paths = {"LL": {"NCCL_PROTO": "LL"}, "DIRECT": {"NCCL_PROTO": "Simple"}}
    if coll == "reducescatter":
        paths.update({"LL128": {"NCCL_PROTO": "LL128"},
                      "DIRECT_PULLS": {"NCCL_PROTO": "Simple", "NCCL_AMD_AG_PULL": "1", "NCCL_AMD_RS_PULL": "1"},
                      "DIRECT_PUSH": {"NCCL_PROTO": "Simple", "NCCL_AMD_AG_PULL": "0"},
                      "REGISTERED": {"NCCL_PROTO": "Simple"}})
    results = {}
    for name, env in paths.items():
        for k in ("NCCL_PROTO", "NCCL_AMD_AG_PULL", "NCCL_AMD_RS_PULL"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        comms = nccl_amd.Communicator.init_all([0, 0, 0])
        streams = [torch.cuda.Stream() for _ in range(3)]
        out = {}
        for op in (0, 1, 2, 3, 4):
            ins = _with_specials(G.make_inputs(3, dtype, count, seed=31 + op), dtype)
            bufs = [torch.from_numpy(np.ascontiguousarray(x).view(vt).copy()).cuda() for x in ins]
            outs = [torch.zeros(per if coll == "reducescatter" else count, dtype=bufs[0].dtype, device="cuda")
                    for _ in bufs]
            hs = ([(c, c.register_buffer(b.data_ptr(), b.numel() * es)) for c, b in zip(comms, bufs)] +
                  [(c, c.register_buffer(o.data_ptr(), o.numel() * es)) for c, o in zip(comms, outs)]
                  if name == "REGISTERED" else [])
            torch.cuda.synchronize()
            with nccl_amd.group():
                for r, (c, st) in enumerate(zip(comms, streams)):
                    if coll == "reducescatter":
                        c.reduce_scatter_raw(bufs[r].data_ptr(), outs[r].data_ptr(), per, dtype, op, st.cuda_stream)
                    else:
                        c.reduce_raw(bufs[r].data_ptr(), outs[r].data_ptr(), count, dtype, op, 1, st.cuda_stream)
            torch.cuda.synchronize()
            out[op] = {r: outs[r].cpu().numpy() for r in (range(3) if coll == "reducescatter" else [1])}
            for c, h in hs:
                c.deregister_buffer(h)
        for c in comms:
            c.destroy()
        results[name] = out
    errs = []
    for op in (0, 1, 2, 3, 4):
        keep = _comparable(_with_specials(G.make_inputs(3, dtype, count, seed=31 + op), dtype), dtype, op)
        for name, out in results.items():
            for r, b in out[op].items():
                k = keep[r * per:(r + 1) * per] if coll == "reducescatter" else keep
                a = results["LL"][op][r]
                if not np.array_equal(a[k], b[k]):
                    bad = np.nonzero(a[k] != b[k])[0]
                    errs.append(f"{coll} {name} vs LL, op {op}, rank {r}: {bad.size} elements differ, e.g. "
                                f"{hex(int(b[k][bad[0]]))} vs {hex(int(a[k][bad[0]]))}")
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("algo", ["RING", "TREE", "REF_ORDER"])
def test_reference_algorithms_with_specials(built, monkeypatch, algo):
    """NaN / +-Inf / +-0 / subnormal / max-finite inputs through the reference's ring and chain (pipe.h) and the
    reference-partition direct kernel, every float type and operator, vs the oracle's ring / chain / partition fold
    (signed zeros compared bitwise, NaN positions)."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    monkeypatch.setenv("NCCL_MULTI_RANK_GPU_ENABLE", "1")
    if algo == "REF_ORDER":
        monkeypatch.setenv("NCCL_AMD_REF_ORDER", "1")
    else:
        monkeypatch.setenv("NCCL_ALGO", algo)
    monkeypatch.setenv("NCCL_BUFFSIZE", "16384")
    monkeypatch.setenv("NCCL_MAX_CTAS", "5")
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0, 0])
    cs = list(zip(comms, [torch.cuda.Stream() for _ in range(3)]))
    errs = []
    for dtype in (7, 8, 6, 9, 10, 11):
        es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
        count = 200_000 // es + 5
        for op in (0, 1, 2, 3, 4):
            ins = _with_specials(G.make_inputs(3, dtype, count, seed=41 + op), dtype)
            errs += G.run_case(cs, "allreduce", dtype, op, count, 0, seed=0, inputs=ins,
                               algo="" if algo == "REF_ORDER" else algo)
            if op in (0, 1, 4):  # and the single-NaN elements bit for bit
                errs += _single_nan_errors(comms, [st for _, st in cs], dtype, count, op, 41 + op,
                                           "" if algo == "REF_ORDER" else algo)
        if errs:
            break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("dtype", [7, 9, 11, 1])
def test_execution_modes_same_bits(built, monkeypatch, dtype):
    """One AllReduce, the same special-value inputs, five ways: eager out of place (the reference), in place, inside a
    group next to a second op (the batched kernel), on symmetric-window buffers (the zero-copy pull kernel), and from
    misaligned base pointers — identical bits, NaN included (outside the elements where two NaNs meet in an add or
    multiply), at an LL size and at a staged size. (hipGraph replay: test_gpu_api.py.)"""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    monkeypatch.setenv("NCCL_MULTI_RANK_GPU_ENABLE", "1")
    torch.cuda.set_device(0)
    n = 3
    es = np.dtype(G.oracle.NP_STORAGE[dtype]).itemsize
    vt = _int_view(dtype)
    comms = nccl_amd.Communicator.init_all([0] * n)
    streams = [torch.cuda.Stream() for _ in range(n)]
    WIN = 8 << 20
    wbufs = [torch.zeros(WIN, dtype=torch.uint8, device="cuda") for _ in range(n)]
    with nccl_amd.group():
        wins = [c.register_window(b.data_ptr(), WIN) for c, b in zip(comms, wbufs)]
    errs = []
    for count in (2048 // es * 3 + 1, 3_000_000 // es):
        for op in (0, 1, 2, 3, 4):
            ins = _with_specials(G.make_inputs(n, dtype, count, seed=51 + op), dtype) if dtype != 1 else \
                G.make_inputs(n, dtype, count, seed=51 + op)
            host = [np.ascontiguousarray(x).view(vt) for x in ins]

            def dev(x, extra=0):
                t = torch.zeros(x.size + extra, dtype=torch.from_numpy(x[:1]).dtype, device="cuda")
                t[extra:].copy_(torch.from_numpy(x.copy()))
                return t

            def run(mode):
                sends = [dev(h) for h in host]
                recvs = [torch.zeros_like(t) for t in sends]
                sp = [t.data_ptr() for t in sends]
                rp = [t.data_ptr() for t in recvs]
                if mode == "inplace":
                    rp = sp
                if mode == "misaligned":  # a base 1 element past a 16-byte boundary on every rank
                    sends = [dev(h, 1) for h in host]
                    recvs = [torch.zeros_like(t) for t in sends]
                    sp = [t.data_ptr() + es for t in sends]
                    rp = [t.data_ptr() + es for t in recvs]
                if mode == "window":
                    for w, h in zip(wbufs, host):
                        w[:h.nbytes].copy_(torch.from_numpy(h.view(np.uint8).copy()))
                    sp = [w.data_ptr() for w in wbufs]
                    rp = [w.data_ptr() + WIN // 2 for w in wbufs]
                extra = [torch.zeros(4096, dtype=torch.float32, device="cuda") for _ in range(n)]
                torch.cuda.synchronize()

                def issue():
                    with nccl_amd.group():
                        for r, (c, st) in enumerate(zip(comms, streams)):
                            c.all_reduce_raw(sp[r], rp[r], count, dtype, op, st.cuda_stream)
                            if mode == "group":
                                c.all_reduce_raw(extra[r].data_ptr(), extra[r].data_ptr(), 4096, 7, 0, st.cuda_stream)
                issue()
                torch.cuda.synchronize()
                if mode == "inplace":
                    return [t.cpu().numpy() for t in sends]
                if mode == "misaligned":
                    return [t.cpu().numpy()[1:] for t in recvs]
                if mode == "window":
                    return [w[WIN // 2:WIN // 2 + count * es].cpu().numpy().view(vt) for w in wbufs]
                return [t.cpu().numpy() for t in recvs]

            ref = run("eager")
            keep = _comparable(ins, dtype, op)
            for mode in ("inplace", "group", "window", "misaligned"):
                got = run(mode)
                for r in range(n):
                    a, b = ref[r][keep], got[r][keep]
                    if not np.array_equal(a, b):
                        bad = np.nonzero(a != b)[0]
                        errs.append(f"count {count} op {op} {mode} rank {r}: {bad.size} differ, e.g. "
                                    f"{hex(int(b[bad[0]]))} vs {hex(int(a[bad[0]]))}")
    with nccl_amd.group():
        for c, w in zip(comms, wins):
            c.deregister_window(w)
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("env", [{"NCCL_AMD_AG_PULL": "1"}, {"NCCL_AMD_RS_PULL": "1", "NCCL_AMD_AG_PULL": "1"},
                                 {"NCCL_AMD_AG_PULL": "1", "NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "2"},
                                 {"NCCL_AMD_AG_PULL": "0", "NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "2"}],
                         ids=["ag_pull", "both_pulls", "ag_pull_tiny_slots", "push_tiny_slots"])
def test_pull_modes_interleaved_with_reduce(built, env):
    """Pull-mode gathers after Reduces on the same communicator: a Reduce pushes to its root only, so the
    per-pair AG sequences diverge; the pull gather must run on its own sequence (found by scripts/fuzz.py:
    an AllGather after a Reduce read a stale slot)."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0, 0])
    finally:
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
    streams = [torch.cuda.Stream() for _ in range(3)]
    cs = list(zip(comms, streams))
    seq = [("reduce", 7, 0, 100_003, 2), ("allgather", 6, 0, 7, 0), ("allreduce", 7, 0, 300_001, 0),
           ("reduce", 2, 3, 50_000, 0), ("reduce", 9, 0, 4099, 1), ("allgather", 7, 0, 70_001, 0),
           ("allreduce", 9, 2, 1_000_003, 0), ("reducescatter", 7, 0, 3 * 40_000, 0), ("allgather", 2, 0, 5, 0)]
    errs = []
    for rep in range(2):
        for i, (coll, dt, op, count, root) in enumerate(seq):
            errs += G.run_case(cs, coll, dt, op, count, 0, seed=1000 * rep + i, root=root)
            if errs:
                break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:10])


def test_multistep_integer_pipelines(built):
    """Multi-step channel pipelines (64 KiB slots, 7 channels) for the 32/64-bit integer kernels: the
    inline-asm write-through stores need their own trailing wait states, or a register reuse right behind a
    store (which register allocation put there for these kernels only) sends pointer-valued garbage in
    16-byte-pack holes. Found by scripts/fuzz.py; bit-exact vs the oracle."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    env = {"NCCL_AMD_SLOT_BYTES": "65536", "NCCL_MAX_CTAS": "7"}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0, 0])
    finally:
        for k, v in saved.items():
            os.environ.pop(k, None)
            if v is not None:
                os.environ[k] = v
    cs = list(zip(comms, [torch.cuda.Stream() for _ in range(3)]))
    errs = []
    for i, (coll, dt, op, count, root) in enumerate([
            ("allreduce", 2, 0, 1 << 20, 0), ("allreduce", 4, 2, 1048587, 0), ("allreduce", 3, 1, 3 << 19, 0),
            ("reduce", 2, 0, 1048587, 1), ("reduce", 4, 2, 1048587, 2), ("reducescatter", 5, 0, 3 << 19, 0),
            ("allgather", 2, 0, 1 << 18, 0)]):
        errs += G.run_case(cs, coll, dt, op, count, 0, seed=4000 + i, root=root)
        if errs:
            break
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:10])


def test_fuzz_short(built):
    """A short randomized sweep (scripts/fuzz.py): random communicator settings x random collectives,
    bit-exact vs the oracle."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "fuzz.py"), "25", "7"],
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-2000:]
    assert "FUZZ OK" in out.stdout


def test_rank_dependent_misalignment(built):
    """Ranks whose buffers are aligned differently must still pick the same protocol and batch (ADVICE r1:
    LL eligibility used to follow each rank's own alignment, so ranks could launch different kernels and
    spin until the timeout). 3 ranks in one process, offsets 0 / 1 / 3 elements, LL and staged sizes."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0, 0])
    cs = list(zip(comms, [torch.cuda.Stream() for _ in comms]))
    errs = []
    for i, (coll, dt, op, count) in enumerate([("allreduce", 7, 0, 1001), ("allreduce", 9, 2, 40_003),
                                               ("allreduce", 6, 0, 3), ("reduce", 2, 3, 5_001),
                                               ("reducescatter", 7, 0, 3 * 2_000), ("allgather", 8, 0, 1_000),
                                               ("allreduce", 7, 0, 700_001), ("reducescatter", 0, 1, 3 * 300)]):
        for mis in ([0, 1, 3], [3, 0, 1], [1, 1, 0]):
            errs += G.run_case(cs, coll, dt, op, count, list(mis), seed=100 + i, root=i % 3)
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("algo,nranks", [("RING", 2), ("RING", 3), ("TREE", 2), ("TREE", 4)])
def test_forced_ring_and_tree(built, algo, nranks, monkeypatch):
    """NCCL_ALGO=RING / TREE run the reference's own algorithms (pipe.h): the ring for AllReduce /
    ReduceScatter / AllGather and the chain to the root for Reduce (RING), the intra-node tree = chain for
    AllReduce (TREE; RS / AG / Reduce fall back to the default plan, as the reference has no tree for them).
    Bit-exact vs the oracle: the ring AllReduce folds in the reference's own partition (channel parts, loops
    of n chunks, oracle_all_reduce_ring_nccl), the chain in oracle_all_reduce_chain's order. Tiny slots force
    many pipeline hops and credit wrap-around; a small NCCL_BUFFSIZE (chunk) many ring loops per channel."""
    torch = _torch()
    import nccl_amd
    from tests import gpu_cases as G
    monkeypatch.setenv("NCCL_MULTI_RANK_GPU_ENABLE", "1")
    monkeypatch.setenv("NCCL_ALGO", algo)
    torch.cuda.set_device(0)
    errs = []
    # (the ring needs >= 2 slots per link, enqueue.cc; the chain also runs with 1)
    for env in ({}, {"NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "2" if algo == "RING" else "1",
                     "NCCL_BUFFSIZE": "16384", "NCCL_MAX_CTAS": "6"}):
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        comms = nccl_amd.Communicator.init_all([0] * nranks)
        cs = list(zip(comms, [torch.cuda.Stream() for _ in comms]))
        for i, (coll, dt, op, count, mis) in enumerate(G.case_list(nranks, quick=True)):
            for root in ([0] if coll != "reduce" else [nranks - 1]):
                errs += G.run_case(cs, coll, dt, op, count, mis, seed=300 + i, root=root, algo=algo)
            if mis == 0 and i % 3 == 0:
                errs += G.run_case(cs, coll, dt, op, count, mis, seed=300 + i, inplace=True, algo=algo)
            if errs:
                break
        for c in comms:
            c.destroy()
        if errs:
            break
    assert not errs, "\n".join(errs[:20])


def _mapcheck_worker(rank, nranks, uid, q, fault_rank, fault):
    try:
        logf = f"/tmp/nccl_amd_mapcheck_{os.getpid()}.log"
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_FILE=logf, NCCL_AMD_SPIN_TIMEOUT_MS="20000")
        if rank == fault_rank:
            # 1: this rank's stores never arrive (the init fails); 2: only in the first round, so the second round's
            # remap through hipIpc handles repairs it; 3: this rank's part of the check fails before its kernel
            os.environ["NCCL_AMD_MAPCHECK_FAULT"] = str(fault)
        import torch
        import nccl_amd
        torch.cuda.set_device(0)
        try:
            comm = nccl_amd.Communicator.init(nranks, rank, uid)
        except nccl_amd.NcclError as e:
            text = open(logf).read() if os.path.exists(logf) else ""
            q.put((rank, ("error", e.code, str(e) + "\n" + text)))
            return
        from tests import gpu_cases as G
        errs = G.run_case([(comm, torch.cuda.Stream())], "allreduce", 7, 0, 100_001, 0, seed=3)
        comm.destroy()
        text = open(logf).read() if os.path.exists(logf) else ""
        q.put((rank, ("ok", "peer mappings verified" in text, errs, "remapped through hipIpc handles" in text)))
    except Exception as e:
        q.put((rank, ("exception", repr(e), [])))


@pytest.mark.parametrize("fault", [0, 1, 2, 3], ids=["clean", "broken", "repaired", "stepfail"])
def test_mapping_check_at_init(built, fault):
    """every communicator init stores a pattern through each peer mapping (staging and flags, the
    kernels' own write-through store) and loads the peers' patterns back before the first collective. Same-device
    here (every rank on the box's one GPU over dma-buf imports). broken: NCCL_AMD_MAPCHECK_FAULT=1 on rank 2 (its
    stores dropped in both rounds, as a broken mapping would) — every rank's init fails together with ncclSystemError
    within seconds, the ranks that saw it naming rank 2 and the failing allocation. repaired: dropped in the first
    round only — rank 2 re-imports its peers through the exports' hipIpc handles, the second round passes and the
    AllReduce is bit-exact on those mappings. stepfail: rank 2's part of the check fails before its kernel — it returns
    that error and its peers ncclRemoteError at once, not after the bootstrap timeout (the failure branches:
    tests/test_mapcheck.py)."""
    import queue
    import time
    _torch()
    import nccl_amd
    uid = nccl_amd.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mapcheck_worker, args=(r, 3, uid, q, 2 if fault else 99, fault)) for r in range(3)]
    t0 = time.time()
    for p in ps:
        p.start()
    res = {}
    while len(res) < 3 and time.time() - t0 < 240:
        try:
            r, out = q.get(timeout=30)
            res[r] = out
        except queue.Empty:
            if not any(p.is_alive() for p in ps):
                break
    for p in ps:
        if p.is_alive():
            p.kill()
        p.join(timeout=60)
    assert len(res) == 3, res
    if fault in (0, 2):
        assert all(o[0] == "ok" and o[1] and not o[2] for o in res.values()), res
        assert res[2][3] == (fault == 2) and not res[0][3] and not res[1][3], res
    elif fault == 1:
        assert all(o[0] == "error" and o[1] == 2 for o in res.values()), res
        for r in (0, 1):
            assert f"rank 2 (device 0" in res[r][2] and "did not arrive" in res[r][2], res[r]
        assert time.time() - t0 < 120
    else:
        assert all(o[0] == "error" for o in res.values()), res
        assert res[2][1] == 1 and res[0][1] == 6 and res[1][1] == 6, res
        for r in (0, 1):
            assert "rank 2 could not run its part of the check" in res[r][2], res[r]
        assert time.time() - t0 < 120
