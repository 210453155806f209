"""Randomized parity fuzzing on the GPU: random communicator settings (ranks 2-4 in one process, slot size,
slot count, channel cap, protocol / algorithm, pull variants) and, per communicator, random collectives
(type, op, count incl. ragged and tiny, misaligned bases, in place, root; sometimes a group of several
collectives, so small AllReduces aggregate into LL batches between other ops; a quarter of the communicators
in symmetric windows, a quarter on ncclCommRegister'd buffers; a quarter with eager registration) checked bit-exact
against the CPU oracle. Usage: python scripts/fuzz.py SECONDS [SEED]. Prints one line per communicator."""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "10000")
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
import torch  # noqa: E402

import nccl_amd  # noqa: E402
from tests import gpu_cases as G  # noqa: E402

KNOBS = ("NCCL_PROTO", "NCCL_ALGO", "NCCL_AMD_SLOT_BYTES", "NCCL_AMD_NSLOTS", "NCCL_MAX_CTAS", "NCCL_AMD_AG_PULL",
         "NCCL_AMD_RS_PULL", "NCCL_AMD_MIN_CHANNEL_BYTES", "NCCL_AMD_LL_CHANNEL_BYTES", "NCCL_AMD_LL128",
         "NCCL_AMD_LL128_CHANNEL_BYTES", "NCCL_AMD_SYM_WT", "NCCL_AMD_P2P_FENCE", "NCCL_AMD_LINK_CHANNELS",
         "NCCL_BUFFSIZE", "NCCL_AMD_REF_ORDER", "NCCL_LL_BUFFSIZE", "NCCL_LL128_BUFFSIZE", "NCCL_AMD_REF_NCHANNELS",
         "NCCL_AMD_EAGER_REGISTER", "NCCL_AMD_EAGER_REGISTER_BYTES", "NCCL_AMD_EAGER_REGISTER_MAX")


def settings(rng):
    env = {}
    if rng.random() < 0.3:
        env["NCCL_PROTO"] = rng.choice(["LL", "^LL", "Simple", "LL,Simple", "LL128", "LL,LL128", "LL128,Simple"])
    if rng.random() < 0.3:
        env["NCCL_ALGO"] = rng.choice(["ONESHOT", "DIRECT", "RING"])
        if env["NCCL_ALGO"] == "RING" and env.get("NCCL_PROTO") == "LL,LL128":
            env["NCCL_PROTO"] = "LL,Simple"  # LL kernel / ring split by capacity (tests/gpu_cases.py ring_runs)
    if rng.random() < 0.4:
        env["NCCL_AMD_SLOT_BYTES"] = str(rng.choice([4096, 8192, 16384, 65536]))
    if rng.random() < 0.3:
        env["NCCL_AMD_NSLOTS"] = str(rng.choice([1, 2, 3]))
    if rng.random() < 0.3:
        env["NCCL_MAX_CTAS"] = str(rng.choice([1, 3, 7, 32, 64]))
    if rng.random() < 0.3:
        env["NCCL_AMD_AG_PULL"] = "0"  # the push gather (pull is the default)
    if rng.random() < 0.3:
        env["NCCL_AMD_RS_PULL"] = "1"
    if rng.random() < 0.2:
        env["NCCL_AMD_MIN_CHANNEL_BYTES"] = str(rng.choice([4096, 16384]))
    if rng.random() < 0.2:
        env["NCCL_AMD_LL_CHANNEL_BYTES"] = str(rng.choice([512, 1024, 8192]))
    if rng.random() < 0.3:  # the LL128 class (64-byte lines) in its size-table range
        env["NCCL_AMD_LL128"] = "1"
    if rng.random() < 0.2:
        env["NCCL_AMD_LL128_CHANNEL_BYTES"] = str(rng.choice([56, 512, 16384]))
    if rng.random() < 0.3:
        env["NCCL_AMD_SYM_WT"] = "0"  # the symmetric kernels' write-back publish instead of write-through
    if rng.random() < 0.3:
        env["NCCL_AMD_P2P_FENCE"] = "1"  # the release fence the cross-device default keeps
    if rng.random() < 0.2:
        env["NCCL_AMD_LINK_CHANNELS"] = str(rng.choice([2, 8, 16]))  # the n >= 3 CU budget, tightened
    if rng.random() < 0.15:  # AllReduce on the direct kernel in the reference's ring partition
        env["NCCL_AMD_REF_ORDER"] = "1"
    if rng.random() < 0.3 and (env.get("NCCL_AMD_REF_ORDER") or env.get("NCCL_ALGO") == "RING"):
        # the reference run's K apart from the channel cap: its parts shared by several workgroups (refSub)
        env["NCCL_AMD_REF_NCHANNELS"] = str(rng.choice([1, 2, 5, 16, 64, 100]))
        if rng.random() < 0.5:
            env["NCCL_AMD_MIN_CHANNEL_BYTES"] = str(rng.choice([512, 1024, 4096]))
    if rng.random() < 0.2:  # the reference's knob: slot size here, and the ring's chunk (many ring loops)
        env["NCCL_BUFFSIZE"] = str(rng.choice([8192, 16384, 65536]))
    if rng.random() < 0.15:  # the LL / LL128 ring chunks REF_ORDER walks when NCCL_PROTO names that protocol alone
        env["NCCL_LL_BUFFSIZE"] = str(rng.choice([4096, 65536, 524288]))
    if rng.random() < 0.15:
        env["NCCL_LL128_BUFFSIZE"] = str(rng.choice([32768, 262144]))
    # eager zero-copy on the cases' plain torch buffers (register.cc), small thresholds too: "1" on, "-1" on across
    # processes only (scripts/fuzz_mp.py; off in this one-process fuzz), "0" or unset off (the default)
    r = rng.random()
    if r < 0.25:
        env["NCCL_AMD_EAGER_REGISTER"] = "-1"
    elif r < 0.5:
        env["NCCL_AMD_EAGER_REGISTER"] = "1"
    if r < 0.5 or rng.random() < 0.5:
        if rng.random() < 0.6:
            env["NCCL_AMD_EAGER_REGISTER_BYTES"] = str(rng.choice([16, 4096, 65536]))
        if rng.random() < 0.3:
            env["NCCL_AMD_EAGER_REGISTER_MAX"] = str(rng.choice([1, 2]))
    return env


def run_window_cases(cs, rng, k, registered=False):
    """k random cases with every buffer inside NCCL_WIN_COLL_SYMMETRIC windows at the same offsets on every
    rank (the symmetric kernels; Reduce and LL-sized ops take their usual paths), or with registered=True in
    buffers registered with ncclCommRegister (the zero-copy kernel in registered mode), checked bit-exact."""
    import numpy as np
    import oracle
    from tests import test_gpu_windows as W
    n = len(cs)
    if registered:
        bufs = [torch.empty(W.WIN_BYTES, dtype=torch.uint8, device="cuda") for _ in cs]
        wins = [c.register_buffer(b.data_ptr(), W.WIN_BYTES) for (c, _), b in zip(cs, bufs)]
    else:
        bufs, wins = W._windows([c for c, _ in cs])
    bases = [(b, b.data_ptr()) for b in bufs]
    errs, done = [], 0
    for _ in range(k):
        coll = rng.choice(["allreduce", "allreduce", "reducescatter", "allgather", "reduce"])
        dt = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
        op = 0 if coll == "allgather" else rng.choice([0, 1, 2, 3, 4])
        es = np.dtype(oracle.NP_STORAGE[dt]).itemsize
        off = rng.choice([0, 0, 0, 1, 3])
        inplace = off == 0 and rng.random() < 0.3
        span = (W.HALF - 64) // es  # elements one half of the window holds past the offset
        count = rng.choice([1, 7, 16, 1000, 4099, 65_536, 100_003, 300_001])
        if coll in ("reducescatter", "allgather"):
            count = min(count, span // n)
            count = max(1, count // n) * n if coll == "reducescatter" else max(1, count)
        count = min(count, span)
        root = rng.randrange(n)
        e = W._run(cs, bases, coll, dt, op, count, off, inplace, seed=rng.randrange(1 << 30), root=root)
        done += 1
        if e:
            errs.append(f"{'registered' if registered else 'window'} {coll} dt={dt} op={op} count={count} off={off} "
                        f"inplace={inplace} root={root}: {e[:3]}")
            break
    for (c, _), w in zip(cs, wins):
        if registered:
            c.deregister_buffer(w)
        else:
            c.deregister_window(w)
    return errs, done


def run_group(cs, ops, rng):
    """Several collectives in ONE group (ops outer, ranks inner: every rank issues the same sequence), so
    runs of small AllReduces aggregate into LL batches between the other ops; every output checked."""
    import numpy as np
    import oracle
    n = len(cs)
    dev = torch.device("cuda", 0)
    plans = []
    for coll, dt, op, count, root in ops:
        ins = G.make_inputs(n, dt, count, rng.randrange(1 << 30))
        exp = G.expected(coll, ins, dt, op, root)
        npdt = oracle.NP_STORAGE[dt]
        bufs = []
        for r in range(n):
            b1, sv = G.to_device(ins[r], dev)
            rv, b2 = None, None
            if coll != "reduce" or r == root:
                b2, rv = G.to_device(np.zeros(G.out_count(coll, n, count), dtype=npdt), dev)
            bufs.append((b1, sv, b2, rv))
        plans.append((coll, dt, op, count, root, exp, npdt, bufs))
    torch.cuda.synchronize()
    with nccl_amd.group():
        for coll, dt, op, count, root, exp, npdt, bufs in plans:
            for (comm, stream), (b1, sv, b2, rv) in zip(cs, bufs):
                G.launch(comm, coll, sv, rv, count, dt, op, root, stream.cuda_stream)
    torch.cuda.synchronize()
    errs = []
    for k, (coll, dt, op, count, root, exp, npdt, bufs) in enumerate(plans):
        for r, (b1, sv, b2, rv) in enumerate(bufs):
            if rv is None:
                continue
            got = G.from_device(rv, npdt)
            want = exp[0] if coll == "reduce" else exp[r]
            if not G.same_bits(got, want, dt):
                errs.append(f"group op {k} {coll} dt={dt} op={op} count={count} root={root} rank {r}: "
                            f"{int((got != want).sum())} mismatches")
    for comm, _ in cs:
        if comm.async_error():
            errs.append(f"rank {comm.rank}: async error {comm.async_error()}")
    return errs


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 60
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rng = random.Random(seed)
    torch.cuda.set_device(0)
    t_end = time.time() + budget
    total, failures = 0, []
    while time.time() < t_end and not failures:
        n = rng.choice([2, 2, 3, 4])
        env = settings(rng)
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(env)
        comms = nccl_amd.Communicator.init_all([0] * n)
        streams = [torch.cuda.Stream() for _ in range(n)]
        cs = list(zip(comms, streams))
        done = 0
        mode = rng.random()
        if mode < 0.5:  # symmetric windows (a quarter) or registered buffers (a quarter) for this communicator
            errs, k = run_window_cases(cs, rng, rng.randint(4, 12), registered=mode >= 0.25)
            total += k
            done += k
            if errs:
                failures.append(f"n={n} env={env} {errs[0]}")
        for _ in range(0 if failures else rng.randint(4, 12)):
            if rng.random() < 0.2:  # a group of several ops: LL batches between other collectives
                dt = rng.choice([2, 6, 7, 9])
                op = rng.choice([0, 2, 3])
                ops = []
                for _k in range(rng.randint(2, 12)):
                    coll = rng.choice(["allreduce"] * 4 + ["reducescatter", "allgather", "reduce"])
                    count = rng.choice([1, 5, 64, 1000, 2048, 4099, 30_000, 200_001])
                    if coll == "reducescatter":
                        count = max(1, count // n) * n
                    ops.append((coll, dt, 0 if coll == "allgather" else op, count, rng.randrange(n)))
                errs = run_group(cs, ops, rng)
                total += len(ops)
                done += len(ops)
                if errs:
                    failures.append(f"n={n} env={env} group {ops}: {errs[:3]}")
                    break
                continue
            coll = rng.choice(["allreduce", "allreduce", "reducescatter", "allgather", "reduce"])
            dt = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
            op = 0 if coll == "allgather" else rng.choice([0, 1, 2, 3, 4])
            count = rng.choice([1, 2, 3, 7, 8, 15, 16, 17, 255, 1000, 4096, 4099, 65_536, 100_003, 1 << 20,
                                (1 << 20) + 11, 3_000_001])
            if coll == "reducescatter":
                count = max(1, count // n) * n
            mis = rng.choice([0, 0, 0, 1, 3])
            inplace = mis == 0 and rng.random() < 0.25
            root = rng.randrange(n)
            seed = rng.randrange(1 << 30)
            ins, special = None, dt in G.FLOAT_TYPES and rng.random() < 0.3
            if special:  # NaN / +-Inf / +-0 / subnormals / max-finite at every 37th element (oracle: NaN positions)
                from tests.test_gpu_collectives import _with_specials
                ins = _with_specials(G.make_inputs(n, dt, count, seed), dt)
            # pinned host buffers on some ranks (the kernels cross PCIe; eager registration falls back to the bounce)
            host = [rng.random() < 0.5 for _ in range(n)] if rng.random() < 0.15 else False
            errs = G.run_case(cs, coll, dt, op, count, mis, seed=seed, inplace=inplace, root=root, inputs=ins,
                              host=host)
            total += 1
            done += 1
            if errs:
                failures.append(f"n={n} env={env} {coll} dt={dt} op={op} count={count} mis={mis} inplace={inplace} "
                                f"root={root} specials={special} host={host}: {errs[:3]}")
                break
        for c in comms:
            c.destroy()
        print(f"n={n} env={env}: {done} cases ok" if not failures else failures[-1], flush=True)
    print(f"FUZZ {'FAIL' if failures else 'OK'}: {total} cases, seed {seed}", flush=True)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
