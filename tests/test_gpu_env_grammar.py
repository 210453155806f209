"""NCCL_ALGO / NCCL_PROTO in the reference's grammar (reference src/graph/tuning.cc:36-136 parseList,
:440-462; docs env.rst:1251-1339) on the GPU: per-function entries pick different kernels for different collectives
of one communicator — seen in the kernel log (NCCL_AMD_KERNEL_LOG) — with every result bit-exact vs the oracle; an
unparsable string fails communicator init with ncclInvalidUsage on every rank; a collective left without an algorithm
available here fails with ncclInvalidUsage (reference enqueue.cc:2052-2065). The planning itself is pinned on the CPU
(tests/test_planning.py test_proto_grammar_*)."""
import multiprocessing as mp
import os
import queue

import pytest

pytestmark = pytest.mark.gpu

# (collective, count as gpu_cases.run_case takes it, kernel-name fragment the collective must launch)
SCENARIOS = {
    # the reference's own example (tuning.cc:49): LL + Simple everywhere, all but LL for AllReduce
    "LL,Simple;allreduce:^LL": ("NCCL_PROTO", [("allreduce", 1024, "collKernel<float, 0, 4>"),     # one-shot
                                               ("reducescatter", 2 * 1000, "::llKernel")]),
    # ring everywhere, the chain (the intra-node tree) for AllReduce
    "ring;allreduce:tree": ("NCCL_ALGO", [("allreduce", 100_000, "pipeKernel<float, 0, 3>"),       # PIPE_CHAIN_AR
                                          ("reducescatter", 2 * 50_000, "pipeKernel<float, 0, 1>")]),  # PIPE_RING_RS
}


def _worker(var, val, cases, q):
    try:
        os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "30000"
        os.environ[var] = val
        klog = f"/tmp/nccl_amd_grammar_kernels_{os.getpid()}.log"
        if os.path.exists(klog):
            os.remove(klog)
        os.environ["NCCL_AMD_KERNEL_LOG"] = klog
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0])
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        cs = list(zip(comms, streams))
        errs, launched = [], []
        for i, (coll, count, _) in enumerate(cases):
            if os.path.exists(klog):
                os.remove(klog)
            errs += G.run_case(cs, coll, 7, 0, count, 0, seed=860 + i)
            torch.cuda.synchronize()
            launched.append(open(klog).read().splitlines() if os.path.exists(klog) else [])
        for c in comms:
            c.destroy()
        q.put((errs, launched))
    except Exception as e:
        q.put(([f"exception {e!r}"], []))


@pytest.mark.parametrize("val", list(SCENARIOS))
def test_per_function_entries_pick_kernels(built, val):
    var, cases = SCENARIOS[val]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(var, val, cases, q))
    p.start()
    try:
        errs, launched = q.get(timeout=240)
    except queue.Empty:
        p.kill()
        raise AssertionError("worker timed out")
    p.join(timeout=60)
    assert not errs, "\n".join(errs[:20])
    for (coll, count, frag), lines in zip(cases, launched):
        assert [ln for ln in lines if frag in ln], f"{var}={val}: {coll} {count} wants {frag}, launched {lines}"


@pytest.mark.parametrize("var,val", [("NCCL_PROTO", "Foo"), ("NCCL_PROTO", "LL,Simple;LL128"),
                                     ("NCCL_ALGO", "bogus:Ring")])
def test_bad_string_fails_init_everywhere(built, monkeypatch, var, val):
    import time
    import torch
    import nccl_amd
    torch.cuda.set_device(0)
    monkeypatch.setenv("NCCL_MULTI_RANK_GPU_ENABLE", "1")
    monkeypatch.setenv(var, val)
    with pytest.raises(nccl_amd.NcclError) as e:       # ncclCommInitAll
        nccl_amd.Communicator.init_all([0, 0])
    assert e.value.code == 5
    # ncclCommInitRank (non-blocking, one thread): both ranks report ncclInvalidUsage through the async error
    uid = nccl_amd.get_unique_id()
    cfg = nccl_amd.Config.default(blocking=0)
    comms = [nccl_amd.Communicator.init(2, r, uid, cfg) for r in range(2)]
    t0 = time.time()
    while any(c.async_error() == 7 for c in comms) and time.time() - t0 < 60:
        time.sleep(0.05)
    assert [c.async_error() for c in comms] == [5, 5]
    for c in comms:
        c.destroy()


def test_no_algorithm_available_fails_the_collective(built, monkeypatch):
    """NCCL_ALGO naming only algorithms an xGMI mesh does not have (NVLS, PAT, CollNet) for AllReduce: the
    communicator initialises, AllReduce fails with ncclInvalidUsage before launching anything, and the other
    collectives still run bit-exact."""
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    torch.cuda.set_device(0)
    monkeypatch.setenv("NCCL_MULTI_RANK_GPU_ENABLE", "1")
    monkeypatch.setenv("NCCL_ALGO", "allreduce:NVLS,PAT")
    comms = nccl_amd.Communicator.init_all([0, 0])
    try:
        x = torch.ones(1000, device="cuda")
        with pytest.raises(nccl_amd.NcclError) as e:
            comms[0].allreduce(x, x, nccl_amd.SUM)
        assert e.value.code == 5
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        errs = G.run_case(list(zip(comms, streams)), "reducescatter", 7, 0, 2 * 5000, 0, seed=870)
        assert not errs, errs
    finally:
        for c in comms:
            c.destroy()
