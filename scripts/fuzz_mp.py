"""Randomized parity fuzzing across PROCESSES (HIP IPC path): N processes on the one GPU follow the same
seeded sequence of communicator settings and collectives (each runs only its own rank) and check their
outputs bit-exact against the oracle. Usage: python scripts/fuzz_mp.py NPROC COMMS [SEED]"""
import multiprocessing as mp
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def worker(rank, n, uids, seed, q):
    try:
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "15000"
        import torch
        import nccl_amd
        from fuzz import KNOBS, settings
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        rng = random.Random(seed)
        s = torch.cuda.Stream()
        total = 0
        for uid in uids:
            env = settings(rng)
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(env)
            comm = nccl_amd.Communicator.init(n, rank, uid)
            if rng.random() < 0.3:  # ncclCommRegister'd buffers: the zero-copy kernel in registered mode
                from tests import test_gpu_windows as W
                import numpy as np
                import oracle
                buf = torch.empty(W.WIN_BYTES, dtype=torch.uint8, device="cuda")
                h = comm.register_buffer(buf.data_ptr(), W.WIN_BYTES)
                for _ in range(rng.randint(3, 8)):
                    coll = rng.choice(["allreduce", "allreduce", "reducescatter", "allgather", "reduce"])
                    dt = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
                    op = 0 if coll == "allgather" else rng.choice([0, 1, 2, 3, 4])
                    es = np.dtype(oracle.NP_STORAGE[dt]).itemsize
                    off = rng.choice([0, 0, 1, 3])
                    inplace = off == 0 and rng.random() < 0.3
                    span = (W.HALF - 64) // es
                    count = rng.choice([1, 7, 1000, 4099, 65_536, 300_001])
                    if coll in ("reducescatter", "allgather"):
                        count = min(count, span // n)
                        count = max(1, count // n) * n if coll == "reducescatter" else max(1, count)
                    count = min(count, span)
                    root = rng.randrange(n)
                    errs = W._run([(comm, s)], [(buf, buf.data_ptr())], coll, dt, op, count, off, inplace,
                                  seed=rng.randrange(1 << 30), root=root)
                    total += 1
                    if errs:
                        comm.destroy()
                        q.put((rank, [f"env={env} registered {coll} dt={dt} op={op} count={count} off={off} "
                                      f"inplace={inplace}: {errs[:2]}"], total))
                        return
                comm.deregister_buffer(h)
            for _ in range(rng.randint(4, 10)):
                coll = rng.choice(["allreduce", "allreduce", "reducescatter", "allgather", "reduce"])
                dt = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
                op = 0 if coll == "allgather" else rng.choice([0, 1, 2, 3, 4])
                count = rng.choice([1, 3, 8, 17, 1000, 4099, 65_536, 100_003, (1 << 20) + 11])
                if coll == "reducescatter":
                    count = max(1, count // n) * n
                mis = rng.choice([0, 0, 1])
                root = rng.randrange(n)
                case_seed = rng.randrange(1 << 30)
                errs = G.run_case([(comm, s)], coll, dt, op, count, mis, seed=case_seed, root=root)
                total += 1
                if errs:
                    comm.destroy()
                    q.put((rank, [f"env={env} {coll} dt={dt} op={op} count={count} mis={mis} root={root}: {errs[:2]}"], total))
                    return
            comm.destroy()
        q.put((rank, [], total))
    except Exception as e:
        q.put((rank, [f"rank {rank} exception {e!r}"], 0))


if __name__ == "__main__":
    import queue
    import nccl_amd
    n, ncomms = int(sys.argv[1]), int(sys.argv[2])
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    uids = [nccl_amd.get_unique_id() for _ in range(ncomms)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, n, uids, seed, q)) for r in range(n)]
    for p in ps:
        p.start()
    res = {}
    while len(res) < n:
        try:
            r, errs, total = q.get(timeout=120)
            res[r] = (errs, total)
        except queue.Empty:
            break
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    bad = [e for r in sorted(res) for e in res[r][0]]
    ok = len(res) == n and not bad
    print(f"FUZZ_MP {'OK' if ok else 'FAIL'}: {n} procs, {ncomms} comms, {sum(t for _, t in res.values())} rank-cases, "
          f"seed {seed}; {bad[:3] if bad else ''}{'' if len(res) == n else f' only {len(res)} ranks reported'}",
          flush=True)
    sys.exit(0 if ok else 1)
