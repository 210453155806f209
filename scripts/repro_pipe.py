"""Repro helper for the ring / chain kernels: single process, NRANKS ranks on the one GPU, NCCL_ALGO from the
environment; runs a few cases and prints each outcome (spin timeout lowered so a stall reports fast)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NCCL_AMD_SPIN_TIMEOUT_MS", "3000")
os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
import torch  # noqa: E402
import nccl_amd  # noqa: E402
from tests import gpu_cases as G  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
algo = os.environ.get("NCCL_ALGO", "")
torch.cuda.set_device(0)
for coll, dt, op, count in [("allreduce", 7, 0, 5), ("allreduce", 7, 0, 70_001), ("allreduce", 7, 0, 4096),
                            ("reducescatter", 7, 0, 2 * 4096), ("allgather", 7, 0, 4096), ("reduce", 7, 0, 4096)]:
    comms = nccl_amd.Communicator.init_all([0] * n)
    cs = list(zip(comms, [torch.cuda.Stream() for _ in comms]))
    try:
        errs = G.run_case(cs, coll, dt, op, count, 0, seed=1, algo=algo)
    except Exception as e:
        errs = [repr(e)]
    print(f"{algo} n={n} {coll} count={count}: {'ok' if not errs else errs[:2]}", flush=True)
    for c in comms:
        try:
            c.destroy()
        except Exception as e:
            print("destroy:", e)

if len(sys.argv) > 2 and sys.argv[2] == "full":
    for env in ({}, {"NCCL_AMD_SLOT_BYTES": "4096", "NCCL_AMD_NSLOTS": "2" if algo == "RING" else "1"}):
        os.environ.update(env)
        comms = nccl_amd.Communicator.init_all([0] * n)
        cs = list(zip(comms, [torch.cuda.Stream() for _ in comms]))
        bad = 0
        for i, (coll, dt, op, count, mis) in enumerate(G.case_list(n, quick=True)):
            for inplace in ((False, True) if mis == 0 and i % 3 == 0 else (False,)):
                try:
                    errs = G.run_case(cs, coll, dt, op, count, mis, seed=300 + i, root=n - 1 if coll == "reduce" else 0,
                                      inplace=inplace, algo=algo)
                except Exception as e:
                    errs = [repr(e)]
                if errs:
                    print(f"FAIL {env} case {i} {coll} dt={dt} op={op} count={count} mis={mis} inplace={inplace}: {errs[:2]}",
                          flush=True)
                    bad += 1
            if bad:
                break
        print(f"{algo} n={n} env={env}: {'ok' if not bad else 'FAILED'}", flush=True)
        for c in comms:
            try:
                c.destroy()
            except Exception as e:
                print("destroy:", e)
        if bad:
            break
