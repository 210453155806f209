"""Parity at the BASELINE configs' real sizes, with the default plan (256 channels, 1 GiB
staging, many pipeline steps per channel) — bit-exact vs the oracle (OpenMP, oracle/nccl_oracle.c):

  C2  ncclAllReduce sum fp32, 256 MiB per rank, 2 processes
  C5  ncclReduce min and max int32, 128 MiB per rank, 8 processes, root 0
  C3  ncclReduceScatter + ncclAllGather bf16, 1 GiB bucket, 8 processes
  C4  ncclAllReduce sum fp16, 8 B .. 256 MiB, 8 processes, with LL, one-shot, direct, ring and tree forced

All ranks share the box's one GPU (one process per rank, HIP-shared staging over the dma-buf transport), so
this checks the engine's arithmetic, fold order and protocol at full size, not xGMI. Inputs are the
BASELINE.md §3 splitmix64 sequences (oracle.fill / fill_at); each process generates only what it checks."""
import multiprocessing as mp
import os
import queue
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MIB = 1 << 20


def _seed(r):
    return 0x5EED0000 + r


def _run_ranks(target, nranks, args=(), limit_s=600):
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
            r, errs = q.get(timeout=20)
            results[r] = errs
        except queue.Empty:
            print(f"[{target.__name__}] {len(results)}/{nranks} done, {time.time() - t0:.0f}s", flush=True)
            if not any(p.is_alive() for p in ps):
                break
    for p in ps:
        if p.is_alive() and len(results) < nranks:
            p.kill()
        p.join(timeout=60)
    assert len(results) == nranks, f"only {len(results)} of {nranks} ranks reported"
    bad = [e for r in sorted(results) for e in results[r]]
    assert not bad, "\n".join(bad[:20])


def _setup(rank, nranks, uid, env=None):
    os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "60000"
    os.environ.update(env or {})
    import torch
    import nccl_amd
    torch.cuda.set_device(0)
    return torch, nccl_amd, nccl_amd.Communicator.init(nranks, rank, uid)


def _cmp(tag, got, want, dtype):
    from tests import gpu_cases as G
    if G.same_bits(got, want, dtype):
        return []
    bad = np.nonzero(got != want)[0]
    return [f"{tag}: {bad.size} mismatches of {want.size}, first {bad[:5].tolist()}"]


def _dev(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8)).cuda()


def test_c1_allreduce_fp32_64MiB_n1(built):
    """C1: ncclAllReduce sum fp32, 64 MiB, world_size 1 (reference taskAppend -> ncclLaunchOneRank,
    src/enqueue.cc:3039-3041; src/device/onerank.cu:49-110): out of place the output is the input bit for bit
    (oracle.all_reduce of one rank), in place the call moves nothing and leaves the buffer untouched. Also the
    avg (PreMulSum by 1/1 = identity) at the same size, which takes the one-rank kernel instead of the copy."""
    import oracle
    import torch
    import nccl_amd
    torch.cuda.set_device(0)
    comm = nccl_amd.Communicator.init_all([0])[0]
    try:
        count = 64 * MIB // 4
        src = oracle.fill(7, _seed(0), count)
        want = oracle.all_reduce([src], 7, 0)
        assert want.view(np.uint32).tobytes() == src.view(np.uint32).tobytes()
        send = _dev(torch, src)
        recv = torch.full_like(send, 0xA5)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        comm.all_reduce_raw(send.data_ptr(), recv.data_ptr(), count, 7, 0, s.cuda_stream)
        s.synchronize()
        assert comm.async_error() == 0
        assert not _cmp("C1 out of place", recv.cpu().numpy().view(np.float32), want, 7)
        assert not _cmp("C1 sendbuff", send.cpu().numpy().view(np.float32), src, 7)  # input not written
        # in place: no bytes move (reference onerank.cu:52-56 skips the copy), the buffer is unchanged
        comm.all_reduce_raw(send.data_ptr(), send.data_ptr(), count, 7, 0, s.cuda_stream)
        s.synchronize()
        assert not _cmp("C1 in place", send.cpu().numpy().view(np.float32), src, 7)
        # avg on one rank: PreMulSum by fp32(1/1) = x * 1.0, bit-exact identity (oracle restates it)
        recv.fill_(0)
        torch.cuda.synchronize()
        comm.all_reduce_raw(send.data_ptr(), recv.data_ptr(), count, 7, 4, s.cuda_stream)
        s.synchronize()
        assert not _cmp("C1 avg", recv.cpu().numpy().view(np.float32), oracle.all_reduce([src], 7, 4), 7)
    finally:
        comm.destroy()


def _c2_worker(rank, nranks, uid, q):
    try:
        import oracle
        torch, nccl_amd, comm = _setup(rank, nranks, uid)
        count = 256 * MIB // 4
        inputs = [oracle.fill(7, _seed(r), count) for r in range(nranks)]
        want = oracle.all_reduce(inputs, 7, 0)
        send = _dev(torch, inputs[rank])
        recv = torch.zeros_like(send)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()  # buffers are filled on the default stream; the collective runs on s
        comm.all_reduce_raw(send.data_ptr(), recv.data_ptr(), count, 7, 0, s.cuda_stream)
        s.synchronize()
        errs = [f"rank {rank}: async {comm.async_error()}"] if comm.async_error() else []
        errs += _cmp(f"C2 rank {rank}", recv.cpu().numpy().view(np.float32), want, 7)
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


def test_c2_allreduce_fp32_256MiB_n2(built):
    _run_ranks(_c2_worker, 2)


def _c5_worker(rank, nranks, uid, q):
    try:
        import oracle
        torch, nccl_amd, comm = _setup(rank, nranks, uid)
        count = 128 * MIB // 4
        send = _dev(torch, oracle.fill(2, _seed(rank), count))
        recv = torch.zeros_like(send) if rank == 0 else None
        s = torch.cuda.Stream()
        errs = []
        inputs = [oracle.fill(2, _seed(r), count) for r in range(nranks)] if rank == 0 else None
        torch.cuda.synchronize()
        for name, op in (("min", 3), ("max", 2)):
            comm.reduce_raw(send.data_ptr(), recv.data_ptr() if recv is not None else None, count, 2, op, 0,
                            s.cuda_stream)
            s.synchronize()
            if comm.async_error():
                errs.append(f"rank {rank}: async {comm.async_error()}")
                break
            if rank == 0:
                errs += _cmp(f"C5 {name}", recv.cpu().numpy().view(np.int32), oracle.reduce(inputs, 2, op, 0), 2)
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


def test_c5_reduce_int32_minmax_128MiB_n8(built):
    _run_ranks(_c5_worker, 8)


def _c3_worker(rank, nranks, uid, q):
    try:
        import oracle
        torch, nccl_amd, comm = _setup(rank, nranks, uid)
        total = 1024 * MIB // 2          # bf16 elements in the 1 GiB bucket
        rc = total // nranks
        s = torch.cuda.Stream()
        errs = []
        # ReduceScatter: my whole bucket in, my block out; expected = the fold of every rank's block `rank`
        # in the reference's order rank+1, ..., rank (= a Reduce of those slices to root `rank`)
        send = _dev(torch, oracle.fill(9, _seed(rank), total))
        shard = torch.zeros(rc * 2, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # the zero-fill runs on the default stream: it must not race the collective
        comm.reduce_scatter_raw(send.data_ptr(), shard.data_ptr(), rc, 9, 0, s.cuda_stream)
        s.synchronize()
        slices = [oracle.fill_at(9, _seed(r), rank * rc, rc) for r in range(nranks)]
        errs += _cmp(f"C3 RS rank {rank}", shard.cpu().numpy().view(np.uint16), oracle.reduce(slices, 9, 0, rank), 9)
        del send, slices
        # AllGather: rank q contributes its own synthetic shard; every rank must end with all of them in order
        mine = _dev(torch, oracle.fill(9, _seed(100 + rank), rc))
        full = torch.zeros(total * 2, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        comm.all_gather_raw(mine.data_ptr(), full.data_ptr(), rc, 9, s.cuda_stream)
        s.synchronize()
        want = np.concatenate([oracle.fill(9, _seed(100 + r), rc) for r in range(nranks)])
        errs += _cmp(f"C3 AG rank {rank}", full.cpu().numpy().view(np.uint16), want, 9)
        if comm.async_error():
            errs.append(f"rank {rank}: async {comm.async_error()}")
        comm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


def test_c3_reducescatter_allgather_bf16_1GiB_n8(built):
    _run_ranks(_c3_worker, 8)


C4_SIZES = [8, 4096 + 2, 64 << 10, (1 << 20) + 6, 16 << 20, 256 << 20]
# The reference-partition columns run the reference's K = 32 channel parts, shared by several workgroups each
# (NCCL_AMD_REF_NCHANNELS, the channel cap left at its default: CollArgs::refSub), and REFORDER_CAP32 with one
# workgroup per part (NCCL_MAX_CTAS = 32).
C4_ALGOS = {"LL": {"NCCL_PROTO": "LL"}, "ONESHOT": {"NCCL_ALGO": "ONESHOT", "NCCL_PROTO": "Simple"},
            "DIRECT": {"NCCL_ALGO": "DIRECT", "NCCL_PROTO": "Simple"},
            "RING": {"NCCL_ALGO": "RING", "NCCL_AMD_REF_NCHANNELS": "32"},
            "REFORDER": {"NCCL_AMD_REF_ORDER": "1", "NCCL_AMD_REF_NCHANNELS": "32"},
            "REFORDER_CAP32": {"NCCL_AMD_REF_ORDER": "1", "NCCL_MAX_CTAS": "32"},
            # the reference's RING/LL and RING/LL128 partitions (the lower end of the curve), up to 16 MiB
            "REFORDER_LL": {"NCCL_AMD_REF_ORDER": "1", "NCCL_AMD_REF_NCHANNELS": "32", "NCCL_PROTO": "LL"},
            "REFORDER_LL128": {"NCCL_AMD_REF_ORDER": "1", "NCCL_AMD_REF_NCHANNELS": "32", "NCCL_PROTO": "LL128"},
            "TREE": {"NCCL_ALGO": "TREE"}}
C4_PROTO_MAX = 16 << 20


def _c4_worker(rank, nranks, uid, q, uids):
    try:
        import oracle
        torch, nccl_amd, comm = _setup(rank, nranks, uid)
        comm.destroy()
        errs = []
        s = torch.cuda.Stream()
        comms = {}
        for k, (name, env) in enumerate(C4_ALGOS.items()):  # knobs are read at init: one comm per column
            for key in ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MAX_CTAS", "NCCL_AMD_REF_ORDER", "NCCL_AMD_REF_NCHANNELS"):
                os.environ.pop(key, None)
            os.environ.update(env)
            comms[name] = nccl_amd.Communicator.init(nranks, rank, uids[k])
        for nbytes in C4_SIZES:
            count = nbytes // 2
            inputs = [oracle.fill(6, _seed(r) + nbytes, count) for r in range(nranks)]
            # RING: the reference's ring partition on the RING communicator's 32 channels (enqueue.cc ringParts)
            want = {"direct": oracle.all_reduce(inputs, 6, 0), "chain": oracle.all_reduce_chain(inputs, 6, 0),
                    "ring": oracle.all_reduce_ring_nccl(inputs, 6, 0, 32)}
            if nbytes <= C4_PROTO_MAX:
                want["REFORDER_LL"] = oracle.all_reduce_ring_nccl(inputs, 6, 0, 32, 0, oracle.PROTO_LL)
                want["REFORDER_LL128"] = oracle.all_reduce_ring_nccl(inputs, 6, 0, 32, 0, oracle.PROTO_LL128)
            send = _dev(torch, inputs[rank])
            for name, cm in comms.items():
                if name == "LL" and nbytes > 512 << 10:  # beyond the LL line area the default plan runs
                    continue
                if name.startswith("REFORDER_") and nbytes > C4_PROTO_MAX:
                    continue
                recv = torch.zeros_like(send)
                torch.cuda.synchronize()
                cm.all_reduce_raw(send.data_ptr(), recv.data_ptr(), count, 6, 0, s.cuda_stream)
                s.synchronize()
                if cm.async_error():
                    errs.append(f"{name} {nbytes} B rank {rank}: async {cm.async_error()}")
                    break
                errs += _cmp(f"C4 {name} {nbytes} B rank {rank}", recv.cpu().numpy().view(np.uint16),
                             want[name] if name in want else
                             want["chain" if name == "TREE" else "ring" if name in ("RING", "REFORDER", "REFORDER_CAP32")
                                  else "direct"], 6)
            if errs:
                break
        for cm in comms.values():
            cm.destroy()
        q.put((rank, errs))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


def test_c4_allreduce_fp16_sweep_every_algorithm_n8(built):
    import nccl_amd
    uids = [nccl_amd.get_unique_id() for _ in C4_ALGOS]
    _run_ranks(_c4_worker, 8, args=(uids,), limit_s=900)
