"""Randomized parity fuzzing on the GPU: random communicator settings (ranks 2-4 in one process, slot size,
slot count, channel cap, protocol / algorithm, pull variants) and, per communicator, random collectives
(type, op, count incl. ragged and tiny, misaligned bases, in place, root, grouped batches) checked bit-exact
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
         "NCCL_AMD_RS_PULL", "NCCL_AMD_MIN_CHANNEL_BYTES", "NCCL_AMD_LL_CHANNEL_BYTES")


def settings(rng):
    env = {}
    if rng.random() < 0.3:
        env["NCCL_PROTO"] = rng.choice(["LL", "^LL", "Simple", "LL,Simple"])
    if rng.random() < 0.3:
        env["NCCL_ALGO"] = rng.choice(["ONESHOT", "DIRECT", "RING"])
    if rng.random() < 0.4:
        env["NCCL_AMD_SLOT_BYTES"] = str(rng.choice([4096, 8192, 16384, 65536]))
    if rng.random() < 0.3:
        env["NCCL_AMD_NSLOTS"] = str(rng.choice([1, 2, 3]))
    if rng.random() < 0.3:
        env["NCCL_MAX_CTAS"] = str(rng.choice([1, 3, 7, 32, 64]))
    if rng.random() < 0.3:
        env["NCCL_AMD_AG_PULL"] = "1"
    if rng.random() < 0.3:
        env["NCCL_AMD_RS_PULL"] = "1"
    if rng.random() < 0.2:
        env["NCCL_AMD_MIN_CHANNEL_BYTES"] = str(rng.choice([4096, 16384]))
    if rng.random() < 0.2:
        env["NCCL_AMD_LL_CHANNEL_BYTES"] = str(rng.choice([512, 1024, 8192]))
    return env


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
        for _ in range(rng.randint(4, 12)):
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
            errs = G.run_case(cs, coll, dt, op, count, mis, seed=rng.randrange(1 << 30), inplace=inplace, root=root)
            total += 1
            done += 1
            if errs:
                failures.append(f"n={n} env={env} {coll} dt={dt} op={op} count={count} mis={mis} inplace={inplace} "
                                f"root={root}: {errs[:3]}")
                break
        for c in comms:
            c.destroy()
        print(f"n={n} env={env}: {done} cases ok" if not failures else failures[-1], flush=True)
    print(f"FUZZ {'FAIL' if failures else 'OK'}: {total} cases, seed {seed}", flush=True)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
