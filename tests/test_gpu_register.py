"""GPU parity tests of zero-copy collectives on buffers registered with ncclCommRegister (reference
src/register/register.cc:154-200, src/register/coll_reg.cc:326-395; docs/userguide/source/usage/bufferreg.rst:
every rank registers the buffers it passes). Registration is local: the allocation is mapped into every peer
process by that peer's fd server (ipc.cc IMPORT), and the collective runs the symmetric kernel in registered
mode — the peers' buffer addresses are exchanged by the kernels at entry (kernels.h symKernel regMode, the
reference's ptrExchange, prims_simple.h:748-846), so ranks need not use the same offsets. Results must be
bit-identical to the oracle for AllReduce, ReduceScatter and AllGather; Reduce keeps the staged path. Also:
buffers of captured collectives are registered automatically (NCCL_GRAPH_REGISTER, reference enqueue.cc:283).
All ranks share the box's one GPU (single process: raw pointers; multi-process: dma-buf IPC)."""
import multiprocessing as mp
import os
import queue
import re
import time

import numpy as np
import pytest

from tests.test_gpu_windows import HALF, WIN_BYTES, _cases, _run

os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "30000")
pytestmark = pytest.mark.gpu


def _spawn(target, nranks, args=(), limit_s=600):
    import nccl_amd
    uid = nccl_amd.get_unique_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, nranks, uid, q) + tuple(args)) for r in range(nranks)]
    for p in ps:
        p.start()
    results, t0 = {}, time.time()
    while len(results) < nranks and time.time() - t0 < limit_s:
        try:
            r, out = q.get(timeout=20)
            results[r] = out
        except queue.Empty:
            print(f"[{target.__name__}] {len(results)}/{nranks} done, {time.time() - t0:.0f}s", flush=True)
            if not any(p.is_alive() for p in ps):
                break
    for p in ps:
        if p.is_alive() and len(results) < nranks:
            p.kill()
        p.join(timeout=60)
    assert len(results) == nranks, f"only {len(results)} of {nranks} ranks reported"
    return results


def _trace_env(tag):
    logf = f"/tmp/nccl_amd_reg_{tag}_{os.getpid()}.log"
    os.environ["NCCL_DEBUG"] = "TRACE"
    os.environ["NCCL_DEBUG_FILE"] = logf
    return logf


def _zero_copy_lines(logf, pos=0):
    if not os.path.exists(logf):
        return []
    with open(logf) as f:
        f.seek(pos)
        return re.findall(r"(AllReduce|ReduceScatter|AllGather): registered zero-copy", f.read())


@pytest.mark.parametrize("nranks", [2, 3])
def test_registered_single_process(built, nranks, monkeypatch):
    """ncclCommInitAll ranks on one GPU: each registers its whole buffer (ncclCommRegister only, no window);
    every case of the window suite — 13 type/op pairs, ragged counts, in place, unaligned — bit-exact."""
    import torch
    import nccl_amd
    monkeypatch.setenv("NCCL_PROTO", "^LL")
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0] * nranks)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    bufs = [torch.empty(WIN_BYTES, dtype=torch.uint8, device="cuda") for _ in comms]
    handles = [c.register_buffer(b.data_ptr(), WIN_BYTES) for c, b in zip(comms, bufs)]
    cs = list(zip(comms, streams))
    errs = []
    for i, case in enumerate(_cases(nranks, quick=nranks > 2)):
        errs += _run(cs, [(b, b.data_ptr()) for b in bufs], *case, seed=i, root=i % nranks)
        if errs:
            break
    for c, h in zip(comms, handles):
        c.deregister_buffer(h)
    # after deregistration the same buffers take the staged path, still bit-exact
    if not errs:
        errs += _run(cs, [(b, b.data_ptr()) for b in bufs], "allreduce", 7, 0, 200_003, 0, False, seed=99)
    for c in comms:
        c.destroy()
    assert not errs, "\n".join(errs[:20])


def _mp_worker(rank, nranks, uid, q):
    try:
        os.environ["NCCL_PROTO"] = "^LL"
        logf = _trace_env(f"mp{nranks}")
        import torch
        import nccl_amd
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        # a different offset inside the registered allocation on every rank: ranks need not agree on offsets
        shift = 4096 * (rank + 1)
        alloc = torch.empty(WIN_BYTES + 16 * 4096, dtype=torch.uint8, device="cuda")
        buf = alloc[shift:shift + WIN_BYTES]
        h = comm.register_buffer(alloc.data_ptr(), alloc.numel())
        s = torch.cuda.Stream()
        errs = []
        pos = os.path.getsize(logf) if os.path.exists(logf) else 0
        cases = _cases(nranks, quick=True)
        for i, case in enumerate(cases):
            errs += _run([(comm, s)], [(buf, buf.data_ptr())], *case, seed=i, root=i % nranks)
            if errs:
                break
        torch.cuda.synchronize()
        zc = _zero_copy_lines(logf, pos)
        comm.deregister_buffer(h)
        # deregistered: the staged path again, every rank alike
        pos = os.path.getsize(logf)
        if not errs:
            errs += _run([(comm, s)], [(buf, buf.data_ptr())], "allreduce", 7, 0, 100_001, 0, False, seed=77)
        torch.cuda.synchronize()
        after = _zero_copy_lines(logf, pos)
        comm.destroy()
        nonreduce = sum(c[0] != "reduce" for c in cases)
        q.put((rank, (errs, len(zc), nonreduce, len(after))))
    except Exception as e:
        q.put((rank, ([f"rank {rank} exception: {e!r}"], 0, 0, 0)))


@pytest.mark.parametrize("nranks", [2, 4])
def test_registered_multi_process(built, nranks):
    """One process per rank (ncclCommInitRank + dma-buf IPC): ncclCommRegister only. Every AllReduce /
    ReduceScatter / AllGather of the case list runs zero-copy (counted in the NCCL_DEBUG=TRACE plan lines)
    and is bit-exact; the Reduce falls back to the staged path; after ncclCommDeregister the staged path runs."""
    res = _spawn(_mp_worker, nranks)
    bad = [e for r in sorted(res) for e in res[r][0]]
    assert not bad, "\n".join(bad[:20])
    for r, (_, zc, nonreduce, after) in res.items():
        assert zc == nonreduce, f"rank {r}: {zc} zero-copy plans for {nonreduce} eligible collectives"
        assert after == 0, f"rank {r}: zero-copy plan after deregistration"


def _graph_worker(rank, nranks, uid, q):
    """NCCL_GRAPH_REGISTER: a captured AllReduce / ReduceScatter / AllGather registers its buffers itself and
    runs zero-copy on every replay (fresh inputs each time, bit-exact); eager calls on the same buffers keep
    the staged path (automatic registrations serve captures only)."""
    try:
        logf = _trace_env(f"graph{nranks}")
        import torch
        import nccl_amd
        import oracle
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        s = nccl_amd.dedicated_stream(0)
        count = 3 << 20  # 12 MiB fp32: above the one-shot / LL ranges
        x = torch.empty(count, dtype=torch.float32, device="cuda")
        y = torch.empty(count, dtype=torch.float32, device="cuda")
        z = torch.empty(count * nranks, dtype=torch.float32, device="cuda")
        rs = torch.empty(count // nranks, dtype=torch.float32, device="cuda")
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        pos = os.path.getsize(logf) if os.path.exists(logf) else 0
        with torch.cuda.graph(g, stream=s):
            sp = s.cuda_stream
            comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, sp)
            comm.reduce_scatter_raw(x.data_ptr(), rs.data_ptr(), count // nranks, 7, 0, sp)
            comm.all_gather_raw(x.data_ptr(), z.data_ptr(), count, 7, sp)
        zc = _zero_copy_lines(logf, pos)
        errs = []
        for it in range(3):
            ins = G.make_inputs(nranks, 7, count, seed=500 + it)
            x.copy_(torch.from_numpy(ins[rank]))
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                g.replay()
            torch.cuda.synchronize()
            if comm.async_error():
                errs.append(f"rank {rank} replay {it}: async {comm.async_error()}")
                break
            checks = (("allreduce", y, oracle.all_reduce(ins, 7, 0)),
                      ("reducescatter", rs, oracle.reduce_scatter(ins, 7, 0)[rank]),
                      ("allgather", z, oracle.all_gather(ins)))
            for name, out, want in checks:
                if not G.same_bits(out.cpu().numpy(), want, 7):
                    errs.append(f"rank {rank} replay {it}: {name} differs")
        # eager on the same (automatically registered) buffers: staged
        pos = os.path.getsize(logf)
        G.make_inputs(nranks, 7, count, seed=9)
        comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, s.cuda_stream)
        torch.cuda.synchronize()
        eager_zc = _zero_copy_lines(logf, pos)
        del g
        comm.destroy()
        q.put((rank, (errs, len(zc), len(eager_zc))))
    except Exception as e:
        q.put((rank, ([f"rank {rank} exception: {e!r}"], 0, 0)))


def test_graph_register_multi_process(built):
    res = _spawn(_graph_worker, 2)
    bad = [e for r in sorted(res) for e in res[r][0]]
    assert not bad, "\n".join(bad[:20])
    for r, (_, zc, eager) in res.items():
        assert zc == 3, f"rank {r}: {zc} zero-copy plans captured (want 3)"
        assert eager == 0, f"rank {r}: an eager call used an automatic registration"


def _graph_lifetime_worker(rank, nranks, uid, q):
    """Automatic registrations live as long as the graphs that captured them: after the executable graph is destroyed
    (PyTorch already destroyed the hipGraph_t at instantiation), this rank's next blocking call releases them and
    tells the peers (RELEASE), whose own next blocking call unmaps them; a new capture registers the buffers again and
    replays bit-exact."""
    try:
        logf = _trace_env(f"graphlife{nranks}")
        import torch
        import nccl_amd
        import oracle
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        s = nccl_amd.dedicated_stream(0)
        count = 3 << 20
        x = torch.empty(count, dtype=torch.float32, device="cuda")
        y = torch.empty(count, dtype=torch.float32, device="cuda")
        dummy = torch.empty(4096, dtype=torch.uint8, device="cuda")

        def capture_and_check(seed):
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, s.cuda_stream)
            ins = G.make_inputs(nranks, 7, count, seed=seed)
            x.copy_(torch.from_numpy(ins[rank]))
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                g.replay()
            torch.cuda.synchronize()
            ok = not comm.async_error() and G.same_bits(y.cpu().numpy(), oracle.all_reduce(ins, 7, 0), 7)
            return g, ok

        def blocking_call():  # any blocking entry point drains; a registration round trip is one
            h = comm.register_buffer(dummy.data_ptr(), dummy.numel())
            comm.deregister_buffer(h)

        errs = []
        pos0 = os.path.getsize(logf) if os.path.exists(logf) else 0
        g, ok = capture_and_check(700)
        if not ok:
            errs.append(f"rank {rank}: first capture differs")
        held = open(logf).read()[pos0:].count("automatic registration of allocation")
        g.reset()
        torch.cuda.synchronize()
        time.sleep(0.3)
        pos = os.path.getsize(logf)
        blocking_call()  # releases this rank's automatic registrations, RELEASE to the peers
        torch.cuda.synchronize()
        time.sleep(0.3)
        comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), 1024, 7, 0, s.cuda_stream)  # every rank past its release
        torch.cuda.synchronize()
        blocking_call()  # unmaps what the peers released
        text = open(logf).read()[pos:]
        released = text.count("automatic registration of allocation")
        peer_unmaps = sum(int(n) for n in re.findall(r"ipc: released (\d+) peer mapping", text))
        pos = os.path.getsize(logf)
        g2, ok = capture_and_check(701)
        if not ok:
            errs.append(f"rank {rank}: capture after the release differs")
        zc = _zero_copy_lines(logf, pos)
        # the next capture right after the graph is gone, with no blocking call between: the capture itself drops
        # the released references before it looks the buffers up (it must not hand back a registration it frees)
        g2.reset()
        torch.cuda.synchronize()
        time.sleep(0.3)
        g3, ok = capture_and_check(702)
        if not ok:
            errs.append(f"rank {rank}: capture right after the graph's release differs")
        del g3
        comm.destroy()
        q.put((rank, (errs, held, released, peer_unmaps, len(zc))))
    except Exception as e:
        q.put((rank, ([f"rank {rank} exception: {e!r}"], 0, 0, 0, 0)))


def test_graph_registrations_released_with_their_graph(built):
    """graph auto-registrations were kept until communicator destroy. Now a hipUserObject retained by the
    capturing graph drops the reference when the last executable of it is destroyed (register.cc graphHold)."""
    res = _spawn(_graph_lifetime_worker, 2)
    bad = [e for r in sorted(res) for e in res[r][0]]
    assert not bad, "\n".join(bad[:20])
    for r, (_, held, released, peer_unmaps, zc) in res.items():
        assert held == 0, f"rank {r}: a registration was released while its graph lived"
        assert released == 2, f"rank {r}: {released} automatic registrations released (want x and y)"
        # the peer's x and y plus at least its first dummy registration (the dummies alone give at most 2)
        assert peer_unmaps >= 3, f"rank {r}: unmapped {peer_unmaps} of the peer's released buffers (want >= 3)"
        assert zc == 1, f"rank {r}: the re-capture planned {zc} zero-copy AllReduces (want 1)"


def _large_worker(rank, nranks, uid, q):
    """The metric's size on registered buffers: 256 MiB fp32 per rank, every rank's sendbuff and recvbuff in
    separate torch allocations registered with ncclCommRegister, bit-exact vs the oracle at full size."""
    try:
        import torch
        import nccl_amd
        import oracle
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        count = 256 * (1 << 20) // 4
        inputs = [oracle.fill(7, 0x5EED0000 + r, count) for r in range(nranks)]
        want = oracle.all_reduce(inputs, 7, 0)
        send = torch.from_numpy(inputs[rank]).cuda()
        recv = torch.zeros_like(send)
        hs = [comm.register_buffer(send.data_ptr(), send.numel() * 4),
              comm.register_buffer(recv.data_ptr(), recv.numel() * 4)]
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        comm.all_reduce_raw(send.data_ptr(), recv.data_ptr(), count, 7, 0, s.cuda_stream)
        s.synchronize()
        errs = [f"rank {rank}: async {comm.async_error()}"] if comm.async_error() else []
        got = recv.cpu().numpy()
        if not errs and not G.same_bits(got, want, 7):
            bad = np.nonzero(got != want)[0]
            errs.append(f"rank {rank}: {bad.size} mismatches, first {bad[:5].tolist()}")
        for h in hs:
            comm.deregister_buffer(h)
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


def test_registered_allreduce_fp32_256MiB_n2(built):
    res = _spawn(_large_worker, 2)
    bad = [e for r in sorted(res) for e in res[r]]
    assert not bad, "\n".join(bad)


def _dereg_worker(rank, nranks, uid, q):
    """Rank 0 deregisters at once and starts its next (staged) collective; the others deregister later, while
    rank 0's kernel already waits for them. Their release requests reach rank 0's fd server, which must answer
    without waiting for rank 0's device (the unmapping waits for rank 0's next library call, ipc.cc
    ipcDrainReleases): a server that unmapped itself waited in hipFree for rank 0's kernel, which waited for the
    ranks blocked on the server — a stall until the spin timeout (found by scripts/fuzz_mp.py)."""
    try:
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "15000"
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        s = torch.cuda.Stream()
        errs = []
        t0 = time.time()
        for it in range(3):
            buf = torch.empty(WIN_BYTES, dtype=torch.uint8, device="cuda")
            h = comm.register_buffer(buf.data_ptr(), WIN_BYTES)
            errs += _run([(comm, s)], [(buf, buf.data_ptr())], "allreduce", 7, 0, 200_003, 0, False, seed=60 + it)
            torch.cuda.synchronize()
            if rank != 0:
                time.sleep(1.0)
            comm.deregister_buffer(h)
            errs += G.run_case([(comm, s)], "allreduce", 7, 0, 300_001, 0, seed=70 + it)
            if errs or comm.async_error():
                errs.append(f"rank {rank} iteration {it}: async {comm.async_error()}")
                break
        elapsed = time.time() - t0
        comm.destroy()
        q.put((rank, (errs, elapsed)))
    except Exception as e:
        q.put((rank, ([f"rank {rank} exception: {e!r}"], 0)))


def test_deregister_while_peers_run(built):
    res = _spawn(_dereg_worker, 3)
    bad = [e for r in sorted(res) for e in res[r][0]]
    assert not bad, "\n".join(bad[:10])
    assert all(t < 12 for _, t in res.values()), res  # three 1 s delays, no spin timeout


def _dereg_then_new_comm_worker(rank, nranks, uid, q, uid2):
    """bench.py's suite order of round 3 on its own: a symmetric window, then 256 MiB buffers registered with
    ncclCommRegister, deregistered, and at once a NEW communicator allocating, exporting and importing its slab
    and running its first AllReduce. With the peers' mappings torn down on a helper thread meanwhile this failed
    three runs out of three on the one-GPU box (refused dma-buf export, spin timeout, illegal access); mappings are
    now released on the caller's thread at its next library call (ipc.cc ipcDrainReleases)."""
    try:
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "20000"
        import torch
        import nccl_amd
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        s = torch.cuda.current_stream()
        errs = []
        S = 256 << 20
        c = S // 4
        g = torch.Generator(device="cuda")
        want = lambda b: b * (nranks * (nranks + 1) / 2)
        # a symmetric window over a 512 MiB torch allocation (its cached block is what torch hands out next)
        win_t = torch.empty(2 * S, dtype=torch.uint8, device="cuda")
        win = comm.register_window(win_t.data_ptr(), 2 * S)
        g.manual_seed(4321)
        base = torch.randint(-1024, 1025, (c,), device="cuda", generator=g, dtype=torch.int32).float() / 256
        sendw, recvw = win_t[:S].view(torch.float32), win_t[S:].view(torch.float32)
        sendw.copy_(base * (rank + 1))
        for _ in range(3):
            comm.all_reduce_raw(sendw.data_ptr(), recvw.data_ptr(), c, 7, 0, s.cuda_stream)
        torch.cuda.synchronize()
        if not torch.equal(recvw, want(base)):
            errs.append(f"rank {rank}: window AllReduce wrong")
        comm.deregister_window(win)
        del win_t, sendw, recvw, base
        # registered buffers, deregistered
        g.manual_seed(4322)
        base = torch.randint(-1024, 1025, (c,), device="cuda", generator=g, dtype=torch.int32).float() / 256
        sendr = base * (rank + 1)
        recvr = torch.empty_like(sendr)
        hs = [comm.register_buffer(sendr.data_ptr(), S), comm.register_buffer(recvr.data_ptr(), S)]
        for _ in range(5):
            comm.all_reduce_raw(sendr.data_ptr(), recvr.data_ptr(), c, 7, 0, s.cuda_stream)
        torch.cuda.synchronize()
        if not torch.equal(recvr, want(base)):
            errs.append(f"rank {rank}: registered AllReduce wrong")
        for h in hs:
            comm.deregister_buffer(h)
        del sendr, recvr, base
        # at once: a new communicator and its first collectives
        g.manual_seed(4323)
        base = torch.randint(-1024, 1025, (c,), device="cuda", generator=g, dtype=torch.int32).float() / 256
        xs = base * (rank + 1)
        ys = torch.empty_like(xs)
        cm = nccl_amd.Communicator.init(nranks, rank, uid2)
        for _ in range(3):
            cm.all_reduce_raw(xs.data_ptr(), ys.data_ptr(), c, 7, 0, s.cuda_stream)
        torch.cuda.synchronize()
        if cm.async_error() or comm.async_error():
            errs.append(f"rank {rank}: async {comm.async_error()} / {cm.async_error()}")
        elif not torch.equal(ys, want(base)):
            errs.append(f"rank {rank}: the new communicator's AllReduce is wrong")
        cm.destroy()
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


def test_deregistration_then_new_communicator(built):
    import nccl_amd
    res = _spawn(_dereg_then_new_comm_worker, 4, args=(nccl_amd.get_unique_id(),), limit_s=300)
    bad = [e for r in sorted(res) for e in res[r]]
    assert not bad, "\n".join(bad[:10])


def _wait_file(path, limit_s=60):
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > limit_s:
            raise TimeoutError(path)
        time.sleep(0.01)


def _async_after_dereg_worker(rank, nranks, uid, q, tag):
    """a collective issued right after a peer deregistered a buffer returns to the host once its
    work is enqueued (reference nccl.h.in:431-442), even while this rank's previous kernel still waits for that
    peer. Rank 0 issues AllReduce #1 (its kernel waits: rank 1 is deliberately late), rank 1 deregisters (its
    RELEASE request reaches rank 0's fd server), then rank 0 issues AllReduce #2. Round 3 unmapped the peer's
    buffer inside that call with a device-synchronising hipFree, so the call blocked until rank 1 arrived (the
    late rank's delay); the unmapping now waits until none of the library's kernels is in flight when a collective is
    issued (round 6, ipc.cc ipcProgressReleases: AllReduce #1 still is, so #2 leaves it) or for a blocking entry point."""
    try:
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "60000"
        os.environ["NCCL_PROTO"] = "^LL"
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        import oracle
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        s = torch.cuda.Stream()
        errs = []
        reg = torch.empty(WIN_BYTES, dtype=torch.uint8, device="cuda")
        h = comm.register_buffer(reg.data_ptr(), WIN_BYTES)
        errs += _run([(comm, s)], [(reg, reg.data_ptr())], "allreduce", 7, 0, 200_003, 0, False, seed=11)
        torch.cuda.synchronize()
        count = 4 << 20  # 16 MiB fp32: the staged direct kernel
        ins = G.make_inputs(nranks, 7, count, seed=12)
        x = torch.from_numpy(ins[rank]).cuda()
        y1, y2 = torch.empty_like(x), torch.empty_like(x)
        torch.cuda.synchronize()
        flag = lambda name: f"/tmp/nccl_amd_async_{tag}_{name}"
        issue_s = None
        if rank == 0:
            comm.all_reduce_raw(x.data_ptr(), y1.data_ptr(), count, 7, 0, s.cuda_stream)  # waits for rank 1
            open(flag("ar1"), "w").close()
            _wait_file(flag("dereg"))
            t0 = time.time()
            comm.all_reduce_raw(x.data_ptr(), y2.data_ptr(), count, 7, 0, s.cuda_stream)
            issue_s = time.time() - t0
            open(flag("ar2"), "w").close()
        else:
            _wait_file(flag("ar1"))
            comm.deregister_buffer(h)
            h = None
            open(flag("dereg"), "w").close()
            time.sleep(3.0)  # deliberately late
            comm.all_reduce_raw(x.data_ptr(), y1.data_ptr(), count, 7, 0, s.cuda_stream)
            comm.all_reduce_raw(x.data_ptr(), y2.data_ptr(), count, 7, 0, s.cuda_stream)
        s.synchronize()
        if comm.async_error():
            errs.append(f"rank {rank}: async {comm.async_error()}")
        want = oracle.all_reduce(ins, 7, 0)
        for name, y in (("#1", y1), ("#2", y2)):
            if not G.same_bits(y.cpu().numpy(), want, 7):
                errs.append(f"rank {rank}: AllReduce {name} differs")
        if h is not None:
            comm.deregister_buffer(h)
        comm.destroy()
        q.put((rank, (errs, issue_s)))
    except Exception as e:
        q.put((rank, ([f"rank {rank} exception: {e!r}"], None)))


def test_collective_after_peer_deregistration_returns_before_its_kernel(built):
    tag = f"{os.getpid()}_{int(time.time() * 1000)}"
    res = _spawn(_async_after_dereg_worker, 2, args=(tag,), limit_s=300)
    for name in ("ar1", "dereg", "ar2"):
        try:
            os.unlink(f"/tmp/nccl_amd_async_{tag}_{name}")
        except OSError:
            pass
    bad = [e for r in sorted(res) for e in res[r][0]]
    assert not bad, "\n".join(bad[:10])
    issue_s = res[0][1]
    print(f"rank 0: AllReduce #2 issued in {issue_s * 1e3:.2f} ms while its AllReduce #1 waited for the late rank 1")
    assert issue_s < 1.0, f"the collective blocked {issue_s:.2f} s (the late rank's delay is 3 s)"


def _fail_export_worker(rank, nranks, uid, q):
    """rank 1's slab export is refused (NCCL_AMD_IPC_FAIL_EXPORT=1: its peers open a hipIpc handle
    instead), but its fd server still runs and serves registrations: every rank must still take the registered
    zero-copy kernel (one comm-wide decision from the peer table), bit-exact."""
    try:
        if rank == 1:
            os.environ["NCCL_AMD_IPC_FAIL_EXPORT"] = "1"
        os.environ["NCCL_PROTO"] = "^LL"
        logf = _trace_env("failexport")
        import torch
        import nccl_amd
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        buf = torch.empty(WIN_BYTES, dtype=torch.uint8, device="cuda")
        h = comm.register_buffer(buf.data_ptr(), WIN_BYTES)
        s = torch.cuda.Stream()
        pos = os.path.getsize(logf) if os.path.exists(logf) else 0
        errs = _run([(comm, s)], [(buf, buf.data_ptr())], "allreduce", 7, 0, 300_001, 0, False, seed=5)
        torch.cuda.synchronize()
        zc = _zero_copy_lines(logf, pos)
        comm.deregister_buffer(h)
        comm.destroy()
        q.put((rank, (errs, len(zc))))
    except Exception as e:
        q.put((rank, ([f"rank {rank} exception: {e!r}"], 0)))


def test_registration_survives_one_ranks_export_fallback(built):
    res = _spawn(_fail_export_worker, 2)
    bad = [e for r in sorted(res) for e in res[r][0]]
    assert not bad, "\n".join(bad[:10])
    assert all(zc == 1 for _, zc in res.values()), res


def _graph_mismatch_worker(rank, nranks, uid, q):
    """a graph auto-registration that fails on ONE rank (NCCL_AMD_REG_FAIL_EXPORT=1 on rank 1) makes
    that rank capture the staged kernel while rank 0 captures the zero-copy one. The replay must stop on both
    ranks with the kernel-mismatch error (ncclInvalidUsage, kernels.h WaitProbe) well before the spin timeout,
    instead of both waiting for it."""
    try:
        if rank == 1:
            os.environ["NCCL_AMD_REG_FAIL_EXPORT"] = "1"
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "60000"
        os.environ["NCCL_AMD_DESTROY_TIMEOUT_MS"] = "500"
        os.environ["NCCL_PROTO"] = "^LL"
        import torch
        import nccl_amd
        torch.cuda.set_device(0)
        comm = nccl_amd.Communicator.init(nranks, rank, uid)
        s = nccl_amd.dedicated_stream(0)
        count = 3 << 20
        x = torch.ones(count, dtype=torch.float32, device="cuda")
        y = torch.empty_like(x)
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            comm.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, s.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.time()
        with torch.cuda.stream(s):
            g.replay()
        torch.cuda.synchronize()
        elapsed = time.time() - t0
        err = comm.async_error()
        del g
        comm.destroy()
        q.put((rank, ([], err, elapsed)))
    except Exception as e:
        q.put((rank, ([f"rank {rank} exception: {e!r}"], -1, 0)))


def test_graph_registration_failure_on_one_rank_is_reported(built):
    res = _spawn(_graph_mismatch_worker, 2, limit_s=300)
    bad = [e for r in sorted(res) for e in res[r][0]]
    assert not bad, "\n".join(bad[:10])
    for r, (_, err, elapsed) in res.items():
        assert err == 5, f"rank {r}: async error {err} (want ncclInvalidUsage from the mismatch probe)"
        assert elapsed < 20, f"rank {r}: the replay took {elapsed:.1f} s (spin timeout 60 s)"
