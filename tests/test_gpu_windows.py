"""GPU parity tests of the symmetric-window (zero-copy) kernels: ncclCommWindowRegister with
NCCL_WIN_COLL_SYMMETRIC, then AllReduce (two-shot; one-shot when NCCL_AMD_SYM_ONESHOT=1 promises every call
is out of place), ReduceScatter and AllGather whose buffers lie in the windows run kernels.h symKernel, which pulls peers' buffers directly. Results must be
bit-identical to the oracle (same fold order as the staged path). Reduce and non-symmetric windows fall
back to the staged path. All ranks share the box's one GPU (single process: raw pointers; multi-process:
HIP IPC of the window allocations)."""
import multiprocessing as mp
import os

import numpy as np
import pytest

os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "30000")
pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_ll(monkeypatch):
    """Small AllReduce would take the LL protocol (which needs no window); exclude it so the symmetric
    kernels are what these tests exercise."""
    monkeypatch.setenv("NCCL_PROTO", "^LL")

WIN_BYTES = 8 << 20          # per-rank window; send at [0, half), recv at [half, WIN_BYTES)
HALF = WIN_BYTES // 2


def _cases(n, quick=False):
    """(collective, dtype, op, count, elem_offset, inplace)"""
    out = []
    counts = [1, 7, 4096 + 5, 200_003] if not quick else [7, 70_001]
    for dtype, op in ((7, 0), (9, 0), (6, 0), (2, 3), (3, 2), (4, 1), (0, 0), (8, 4), (2, 4), (10, 0), (1, 4),
                      (5, 2), (11, 1)):
        for count in counts:
            out.append(("allreduce", dtype, op, count, 0, False))
        out.append(("reducescatter", dtype, op, 50_001 * n, 0, False))
        out.append(("allgather", dtype, 0, 30_001, 0, False))
    for coll in ("allreduce", "reducescatter", "allgather"):
        out.append((coll, 7, 0, 100_000 * (n if coll == "reducescatter" else 1), 0, True))
        out.append((coll, 7, 0, 64_000 * (n if coll == "reducescatter" else 1), 3, False))  # unaligned
    out.append(("allreduce", 7, 0, 300_000, 0, True))  # large in-place (two-shot even when small)
    out.append(("reduce", 2, 3, 100_003, 0, False))    # no symmetric Reduce: staged fallback
    return out


def _run(comms_streams, bases, coll, dtype, op, count, off, inplace, seed, root=0):
    """bases[i] = device pointer of rank i's window (same layout on every rank)."""
    import torch
    import oracle
    from tests import gpu_cases as G
    n = comms_streams[0][0].nranks
    npdt = oracle.NP_STORAGE[dtype]
    es = np.dtype(npdt).itemsize
    inputs = G.make_inputs(n, dtype, count, seed)
    exp = G.expected(coll, inputs, dtype, op, root)
    ocount = G.out_count(coll, n, count)
    views = []
    for (comm, stream), (base_t, base) in zip(comms_streams, bases):
        r = comm.rank
        raw = base_t.view(torch.uint8)
        send_off = off * es
        recv_off = HALF + off * es
        if inplace:
            recv_off = send_off
        if coll == "allgather" and inplace:
            full = np.zeros(count * n, dtype=npdt)
            full[r * count:(r + 1) * count] = inputs[r]
            raw[recv_off:recv_off + full.nbytes].copy_(torch.from_numpy(full.view(np.uint8).copy()))
            send_ptr = base + recv_off + r * count * es
        else:
            data = np.ascontiguousarray(inputs[r]).view(np.uint8)
            raw[send_off:send_off + data.size].copy_(torch.from_numpy(data.copy()))
            send_ptr = base + send_off
            if not inplace:
                raw[recv_off:recv_off + ocount * es].zero_()
        recv_ptr = base + recv_off
        if coll == "reducescatter" and inplace:
            recv_ptr = base + send_off + r * (count // n) * es
        views.append((comm, stream, send_ptr, recv_ptr, raw, base))
    torch.cuda.synchronize()
    import nccl_amd
    with nccl_amd.group():
        for comm, stream, sp, rp, _, _ in views:
            sid = stream.cuda_stream
            if coll == "allreduce":
                comm.all_reduce_raw(sp, rp, count, dtype, op, sid)
            elif coll == "reducescatter":
                comm.reduce_scatter_raw(sp, rp, count // n, dtype, op, sid)
            elif coll == "allgather":
                comm.all_gather_raw(sp, rp, count, dtype, sid)
            else:
                comm.reduce_raw(sp, rp if comm.rank == root else None, count, dtype, op, root, sid)
    errs = []
    for comm, stream, sp, rp, raw, base in views:
        stream.synchronize()
        if comm.async_error():
            errs.append(f"rank {comm.rank}: async error {comm.async_error()}")
            continue
        if coll == "reduce" and comm.rank != root:
            continue
        start = rp - base  # offset of recv inside the window
        got = raw[start:start + ocount * es].cpu().numpy().view(npdt)
        want = exp[0] if coll == "reduce" else exp[comm.rank]
        if not G.same_bits(got, want, dtype):
            bad = np.nonzero(got != want)[0]
            errs.append(f"rank {comm.rank} {coll} dt={dtype} op={op} count={count} off={off} inplace={inplace}: "
                        f"{bad.size} mismatches, first {bad[:5].tolist()} got {got[bad[:3]].tolist()} "
                        f"want {want[bad[:3]].tolist()}")
    return errs


def _windows(comms, streams_dev=0):
    import torch
    import nccl_amd
    bufs = [torch.empty(WIN_BYTES, dtype=torch.uint8, device=f"cuda:{c.device}") for c in comms]
    with nccl_amd.group():
        wins = [c.register_window(b.data_ptr(), WIN_BYTES) for c, b in zip(comms, bufs)]
    assert all(w.handle for w in wins)
    for c, w, b in zip(comms, wins, bufs):
        assert c.window_user_ptr(w) == b.data_ptr()
    return bufs, wins


@pytest.mark.parametrize("nranks,oneshot,wt", [(2, False, 1), (3, False, 1), (2, True, 1), (2, False, 0), (3, False, 0)])
def test_windows_single_process(built, nranks, oneshot, wt, monkeypatch):
    import torch
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    if oneshot:  # the one-shot window kernel: a rank-uniform promise that every AllReduce is out of place
        monkeypatch.setenv("NCCL_AMD_SYM_ONESHOT", "1")
    # wt=0: the nontemporal-store publish with an L2 write-back release (NCCL_AMD_SYM_WT=0) instead of the
    # default write-through publish
    monkeypatch.setenv("NCCL_AMD_SYM_WT", str(wt))
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0] * nranks)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    bufs, wins = _windows(comms)
    cs = list(zip(comms, streams))
    bases = [(b, b.data_ptr()) for b in bufs]
    errs = []
    for i, case in enumerate(_cases(nranks, quick=nranks > 2)):
        if oneshot and case[5]:
            continue
        errs += _run(cs, bases, *case, seed=i, root=i % nranks)
        if errs:
            break
    for c, w in zip(comms, wins):
        c.deregister_window(w)
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


def test_windows_allgather_mixed_in_place(built):
    """the symmetric AllGather pulls peers' blocks from their OUTPUTS (each rank places its own block
    before entry), so ranks may mix in-place and out-of-place calls and a sendbuff need not lie in a window:
    only the outputs must sit at the same window offset on every rank. (AllReduce / ReduceScatter read
    peers' INPUTS at the caller's own offsets, so they keep NCCL's rule: both buffers at the same offsets.)"""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    n = 3
    comms = nccl_amd.Communicator.init_all([0] * n)
    streams = [torch.cuda.Stream() for _ in range(n)]
    bufs, wins = _windows(comms)
    cs = list(zip(comms, streams))
    errs = []
    cases = [(7, 30_001, [True, False, True], False), (9, 64_000, [False, True, False], False),
             (7, 40_003, [False, False, True], True), (2, 70_000, [True, True, False], True)]
    for i, (dtype, count, mix, outside) in enumerate(cases):
        es = 2 if dtype == 9 else 4
        inputs = G.make_inputs(n, dtype, count, 40 + i)
        want = G.expected("allgather", inputs, dtype, 0, 0)
        sends, ptrs = [], []
        for (c, s), b in zip(cs, bufs):
            r = c.rank
            raw = b.view(torch.uint8)
            raw[HALF:HALF + n * count * es].zero_()
            data = torch.from_numpy(np.ascontiguousarray(inputs[r]).view(np.uint8).copy()).cuda()
            if mix[r]:    # in place: my input is block r of my output
                raw[HALF + r * count * es:HALF + (r + 1) * count * es].copy_(data)
                ptrs.append(b.data_ptr() + HALF + r * count * es)
            elif outside:  # out of place, sendbuff outside any window
                sends.append(data)
                ptrs.append(data.data_ptr())
            else:          # out of place, sendbuff at offset 0 of the window
                raw[:data.numel()].copy_(data)
                ptrs.append(b.data_ptr())
        torch.cuda.synchronize()
        with nccl_amd.group():
            for (c, s), b, sp in zip(cs, bufs, ptrs):
                c.all_gather_raw(sp, b.data_ptr() + HALF, count, dtype, s.cuda_stream)
        for (c, s), b in zip(cs, bufs):
            s.synchronize()
            got = b.view(torch.uint8)[HALF:HALF + n * count * es].cpu().numpy().view(want[c.rank].dtype)
            if not G.same_bits(got, want[c.rank], dtype):
                bad = np.nonzero(got != want[c.rank])[0]
                errs.append(f"case {i} rank {c.rank} mix {mix} outside {outside}: {bad.size} mismatches, "
                            f"first {bad[:5].tolist()}")
    for c, w in zip(comms, wins):
        c.deregister_window(w)
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


def test_window_without_symmetric_flag_uses_staged_path(built):
    import torch
    import nccl_amd
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0])
    streams = [torch.cuda.Stream() for _ in range(2)]
    bufs = [torch.empty(WIN_BYTES, dtype=torch.uint8, device="cuda") for _ in comms]
    with nccl_amd.group():
        wins = [c.register_window(b.data_ptr(), WIN_BYTES, nccl_amd.WIN_DEFAULT) for c, b in zip(comms, bufs)]
    errs = _run(list(zip(comms, streams)), [(b, b.data_ptr()) for b in bufs], "allreduce", 7, 0, 123_457, 0, False, 5)
    h = comms[0].register_buffer(bufs[0].data_ptr(), 1024)
    comms[0].deregister_buffer(h)
    with pytest.raises(nccl_amd.NcclError):
        comms[0].deregister_buffer(h)
    for c, w in zip(comms, wins):
        c.deregister_window(w)
    for c in comms:
        c.destroy()
    assert not errs, errs


def _mp_worker(rank, nranks, uid, q):
    try:
        os.environ["NCCL_PROTO"] = "^LL"
        import torch
        import nccl_amd
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        buf = torch.empty(WIN_BYTES, dtype=torch.uint8, device="cuda")
        win = comm.register_window(buf.data_ptr(), WIN_BYTES)
        s = torch.cuda.Stream()
        errs = []
        for i, case in enumerate(_cases(nranks, quick=True)):
            errs += _run([(comm, s)], [(buf, buf.data_ptr())], *case, seed=i, root=i % nranks)
            if errs:
                break
        comm.deregister_window(win)
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


@pytest.mark.parametrize("nranks", [2, 4])
def test_windows_multi_process(built, nranks):
    import queue
    import time
    import nccl_amd
    uid = nccl_amd.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mp_worker, args=(r, nranks, uid, q)) for r in range(nranks)]
    for p in ps:
        p.start()
    results = {}
    t0 = time.time()
    while len(results) < nranks and time.time() - t0 < 600:
        try:
            r, errs = q.get(timeout=30)
            results[r] = errs
        except queue.Empty:
            if not any(p.is_alive() for p in ps):
                break
    for p in ps:
        if p.is_alive() and len(results) < nranks:
            p.kill()
        p.join(timeout=60)
    assert len(results) == nranks, f"only {len(results)} of {nranks} ranks reported"
    bad = [e for r in sorted(results) for e in results[r]]
    assert not bad, "\n".join(bad[:20])


def _large_worker(rank, nranks, uid, q):
    try:
        os.environ["NCCL_PROTO"] = "^LL"
        import torch
        import nccl_amd
        import oracle
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        win_bytes = 2 << 30                      # one 2 GiB allocation per rank, mapped whole by every peer
        half = win_bytes // 2
        count = half // 4                        # 268,435,456 fp32: 1 GiB in, 1 GiB out
        buf = torch.empty(win_bytes, dtype=torch.uint8, device="cuda")
        win = comm.register_window(buf.data_ptr(), win_bytes)
        inputs = [oracle.fill(7, 0x5EED0000 + r, count) for r in range(nranks)]
        want = oracle.all_reduce(inputs, 7, 0)
        buf[:half].copy_(torch.from_numpy(inputs[rank].view(np.uint8)))
        buf[half:].zero_()
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        comm.all_reduce_raw(buf.data_ptr(), buf.data_ptr() + half, count, 7, 0, s.cuda_stream)
        s.synchronize()
        errs = [] if comm.async_error() == 0 else [f"rank {rank}: async error {comm.async_error()}"]
        got = buf[half:].cpu().numpy().view(np.float32)
        if not errs and not G.same_bits(got, want, 7):
            bad = np.nonzero(got != want)[0]
            errs.append(f"rank {rank}: {bad.size} mismatches in the 1 GiB result, first {bad[:5].tolist()}")
        comm.deregister_window(win)
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


def test_two_gib_window_multi_process(built):
    """DESIGN.md §3 / VERDICT r1 item 1: a 2 GiB window shared between two processes. hipIpcOpenMemHandle
    never returns for allocations of 2 GiB or more in torch's bundled HIP runtime; the dma-buf transport
    (ipc.cc) maps them. Symmetric AllReduce of 1 GiB fp32 per rank, bit-exact vs the oracle."""
    import queue
    import time
    import nccl_amd
    uid = nccl_amd.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_large_worker, args=(r, 2, uid, q)) for r in range(2)]
    for p in ps:
        p.start()
    results = {}
    t0 = time.time()
    while len(results) < 2 and time.time() - t0 < 300:
        try:
            r, errs = q.get(timeout=20)
            results[r] = errs
        except queue.Empty:
            print(f"[two_gib_window] waiting: {len(results)} done, {time.time() - t0:.0f}s", flush=True)
            if not any(p.is_alive() for p in ps):
                break
    for p in ps:
        if p.is_alive() and len(results) < 2:
            p.kill()
        p.join(timeout=60)
    assert len(results) == 2, f"only {len(results)} of 2 ranks reported"
    bad = [e for r in sorted(results) for e in results[r]]
    assert not bad, "\n".join(bad)


def _example_worker(rank, nranks, uid, mode, q):
    """The reference's docs/examples/05_symmetric_memory/01_allreduce/c/main.cc:75-170 (mode "window") and
    04_user_buffer_registration/01_allreduce/c/main.cc:75-166 (mode "register") as written: 1M floats in
    ncclMemAlloc'd buffers, every element = rank, ncclAllReduce sum; every element must be n(n-1)/2."""
    try:
        import ctypes
        import torch
        import nccl_amd
        torch.cuda.set_device(0)
        lib = nccl_amd.load()
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        count = 1024 * 1024
        size = count * 4
        send, recv = ctypes.c_void_p(), ctypes.c_void_p()
        assert lib.ncclMemAlloc(ctypes.byref(send), size) == 0 and lib.ncclMemAlloc(ctypes.byref(recv), size) == 0
        handles = []
        if mode == "window":
            handles = [comm.register_window(send.value, size), comm.register_window(recv.value, size)]
        else:
            handles = [comm.register_buffer(send.value, size), comm.register_buffer(recv.value, size)]
        host = torch.full((count,), float(rank), dtype=torch.float32)
        torch.cuda.synchronize()
        rt = ctypes.CDLL("libamdhip64.so")  # the HIP runtime torch already loaded (matched by soname)
        assert rt.hipMemcpy(send, ctypes.c_void_p(host.data_ptr()), ctypes.c_size_t(size), 1) == 0  # H2D
        s = torch.cuda.Stream()
        comm.all_reduce_raw(send.value, recv.value, count, 7, 0, s.cuda_stream)
        s.synchronize()
        out = torch.empty(count, dtype=torch.float32)
        assert rt.hipMemcpy(ctypes.c_void_p(out.data_ptr()), recv, ctypes.c_size_t(size), 2) == 0  # D2H
        want = float(nranks * (nranks - 1) // 2)
        errs = [] if bool((out == want).all()) else [f"rank {rank} ({mode}): {int((out != want).sum())} elements "
                                                     f"differ from {want}, e.g. {out[:4].tolist()}"]
        for h in handles:
            if mode == "window":
                comm.deregister_window(h)
            else:
                comm.deregister_buffer(h)
        lib.ncclMemFree(send)
        lib.ncclMemFree(recv)
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


@pytest.mark.parametrize("mode,nranks", [("window", 2), ("window", 4), ("register", 3)])
def test_reference_examples_symmetric_and_registered(built, mode, nranks):
    """Known-answer examples of the reference, one process per rank (the MPI examples' layout): the result is
    exact (small integers in fp32) under any fold order, so it pins the windows / registration paths to
    the reference's own expected value, not to the oracle."""
    import queue
    import time
    import nccl_amd
    uid = nccl_amd.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_example_worker, args=(r, nranks, uid, mode, q)) for r in range(nranks)]
    for p in ps:
        p.start()
    results = {}
    t0 = time.time()
    while len(results) < nranks and time.time() - t0 < 240:
        try:
            r, errs = q.get(timeout=20)
            results[r] = errs
        except queue.Empty:
            if not any(p.is_alive() for p in ps):
                break
    for p in ps:
        if p.is_alive() and len(results) < nranks:
            p.kill()
        p.join(timeout=60)
    assert len(results) == nranks, f"only {len(results)} of {nranks} ranks reported"
    bad = [e for r in sorted(results) for e in results[r]]
    assert not bad, "\n".join(bad)
