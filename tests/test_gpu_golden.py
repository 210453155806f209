"""GPU parity against the committed golden fixtures (tests/golden/*.npz, made by make_golden.py from an
independent numpy restatement of the reference's fold order and arithmetic): every fixture runs through
the C ABI with its own rank count — one process per rank, all on the box's one GPU, HIP IPC between
them — under the default size table and with each protocol forced (LL, one-shot, direct), and every
rank's output must match the fixture bit for bit. The NCCL_ALGO=RING fixtures (the reference's full-size ring
partition) run on a ring communicator of their own channel count and NCCL_BUFFSIZE."""
import glob
import multiprocessing as mp
import os
import queue
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))
# protocol settings, each its own communicator (tuning knobs are read at init)
SETTINGS = [{}, {"NCCL_PROTO": "LL"}, {"NCCL_PROTO": "^LL", "NCCL_ALGO": "ONESHOT"},
            {"NCCL_PROTO": "^LL", "NCCL_ALGO": "DIRECT"}]
KNOBS = ("NCCL_PROTO", "NCCL_ALGO", "NCCL_MAX_CTAS", "NCCL_BUFFSIZE", "NCCL_LL_BUFFSIZE", "NCCL_LL128_BUFFSIZE",
         "NCCL_AMD_REF_ORDER", "NCCL_AMD_REF_NCHANNELS", "NCCL_AMD_MIN_CHANNEL_BYTES")
# the protocol a ring fixture's partition belongs to: its NCCL_PROTO value and buffer-size variable
RING_PROTO = {"simple": ("Simple", "NCCL_BUFFSIZE"), "ll": ("LL", "NCCL_LL_BUFFSIZE"),
              "ll128": ("LL128", "NCCL_LL128_BUFFSIZE")}


def _fixtures(n):
    out = []
    for f in FIXTURES:
        z = np.load(f)  # plain arrays only (allow_pickle stays False)
        if int(z["n"]) == n:
            out.append((os.path.basename(f), {k: z[k] for k in z.files}))
    return out


def _ring_settings(z):
    """NCCL_ALGO=RING fixtures (the reference's full-size ring partition) run on communicators of the fixture's
    channel count and protocol buffer size only, with NCCL_PROTO naming the fixture's protocol: the ring kernel
    (NCCL_ALGO=RING) and the direct kernel on the same partition (NCCL_AMD_REF_ORDER=1) — once with one workgroup
    per reference part (NCCL_MAX_CTAS = K) and once with the parts shared by several workgroups (K given as
    NCCL_AMD_REF_NCHANNELS, the channel cap left at its default, 1 KiB sub-chunks allowed so the fixtures' small
    chunks split too; CollArgs::refSub)."""
    proto, var = RING_PROTO[str(z["proto"]) if "proto" in z else "simple"]
    k = str(int(z["nchannels"]))
    buff = {var: str(int(z["buffsize"]))} if int(z["buffsize"]) else {}
    out = []
    for common in ({"NCCL_MAX_CTAS": k}, {"NCCL_AMD_REF_NCHANNELS": k, "NCCL_AMD_MIN_CHANNEL_BYTES": "1024"}):
        common = dict(common, **buff)
        out += [dict(common, NCCL_ALGO="RING", NCCL_PROTO=proto), dict(common, NCCL_AMD_REF_ORDER="1", NCCL_PROTO=proto)]
    return out


def _worker(rank, n, uids, q):
    try:
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "30000"
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        errs = []
        fixtures = _fixtures(n)
        runs = [(setting, [f for f in fixtures if str(f[1]["coll"]) != "allreduce_ring"]) for setting in SETTINGS]
        runs += [(st, [(name, z)]) for name, z in fixtures if str(z["coll"]) == "allreduce_ring" for st in _ring_settings(z)]
        for (setting, fx), uid in zip(runs, uids):
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(setting)
            comm = nccl_amd.Communicator.init(n, rank, uid)
            s = torch.cuda.Stream()
            for name, z in fx:
                coll, dtype, op = str(z["coll"]), int(z["dtype"]), int(z["op"])
                coll = "allreduce" if coll == "allreduce_ring" else coll
                root = int(z["root"]) if "root" in z else 0
                x = z[f"in{rank}"]
                want = z[f"out{rank}"] if coll == "reducescatter" else z["out"]
                keep_in, sv = G.to_device(x, dev)
                rv = None
                if coll != "reduce" or rank == root:
                    keep_out, rv = G.to_device(np.zeros_like(want), dev)
                torch.cuda.synchronize()
                G.launch(comm, coll, sv, rv, x.size, dtype, op, root, s.cuda_stream)
                s.synchronize()
                ae = comm.async_error()
                if ae:
                    errs.append(f"rank {rank} {setting} {name}: async error {ae}")
                    break
                if rv is None:
                    continue
                got = G.from_device(rv, want.dtype)
                if not G.same_bits(got, want, dtype):
                    bad = np.nonzero(got != want)[0]
                    errs.append(f"rank {rank} {setting} {name}: {bad.size} mismatches, first at {bad[:5].tolist()}")
            comm.destroy()
            if errs:
                break
        q.put((rank, errs))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, [f"rank {rank} exception: {e!r}"]))


@pytest.mark.parametrize("n", sorted({int(np.load(f)["n"]) for f in FIXTURES}))
def test_golden_fixtures(built, n):
    import torch
    assert torch.cuda.is_available(), "GPU test on a box without a GPU"
    import nccl_amd
    nring = sum(len(_ring_settings(z)) for _, z in _fixtures(n) if str(z["coll"]) == "allreduce_ring")
    uids = [nccl_amd.get_unique_id() for _ in range(len(SETTINGS) + nring)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, n, uids, q)) for r in range(n)]
    for p in ps:
        p.start()
    results, t0 = {}, time.time()
    while len(results) < n and time.time() - t0 < 600:
        try:
            r, errs = q.get(timeout=30)
            results[r] = errs
        except queue.Empty:
            alive = sum(p.is_alive() for p in ps)
            print(f"[golden n={n}] waiting: {len(results)} done, {alive} alive, {time.time() - t0:.0f}s", flush=True)
            if alive == 0:
                break
    for p in ps:
        if p.is_alive() and len(results) < n:
            p.kill()
    for p in ps:
        p.join(timeout=60)
    assert len(results) == n, f"only {len(results)} of {n} ranks reported"
    bad = [e for r in sorted(results) for e in results[r]]
    assert not bad, "\n".join(bad[:20])
