"""world_size-2 gloo tests (CPU) of the N>1 harness path of bench.py: the ncclUniqueId created by rank 0
(which starts this library's bootstrap root) reaches every rank intact, the max-over-ranks timing, and
the bus-bandwidth arithmetic (reference inspector.cc:1450-1492)."""
import multiprocessing as mp
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        import torch.distributed as dist
        import bench
        dist.init_process_group("gloo", rank=rank, world_size=world)
        uid = bench.exchange_unique_id(dist, rank)
        ids = [None] * world
        dist.all_gather_object(ids, uid)
        same = all(x == ids[0] for x in ids) and len(uid) == 128
        mx = bench.max_over_ranks(dist, [1.0 + rank, 10.0 - rank])
        dist.destroy_process_group()
        q.put((rank, same, mx))
    except Exception as e:
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("world", [2])
def test_gloo_harness(built, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=30)
    for rank, same, mx in res:
        assert same, (rank, mx)
        assert mx == [float(world), 10.0], mx


def test_rates():
    import bench
    S = 256 << 20
    v, alg, bus = bench.rates(8, S, 1.0)
    assert abs(alg - S / 1e-3 / 1e9) < 1e-6
    # at n >= 2 the value IS the metric's busBW (per rank, nccl-tests), not N x busBW
    assert abs(bus - alg * 2 * 7 / 8) < 1e-6 and v == bus
    v2, _, bus2 = bench.rates(2, S, 1.0)
    assert v2 == bus2 and abs(bus2 - S / 1e-3 / 1e9) < 1e-6
    v1, _, bus1 = bench.rates(1, 64 << 20, 1.0)
    assert bus1 == 0 and abs(v1 - 2 * (64 << 20) / 1e-3 / 1e9) < 1e-6
    # the pull gather (default) writes one copy of each reduced block: 3S + 2(n-1)/n S; the push gather 2S + 4(n-1)/n S
    assert bench.hbm_bytes_per_rank("allreduce", 8, S) == int(3 * S + 2 * 7 * S / 8)
    assert bench.hbm_bytes_per_rank("allreduce", 8, S, pull_gather=False) == int(2 * S + 4 * 7 * S / 8)
    assert bench.hbm_bytes_per_rank("allreduce", 2, S) == bench.hbm_bytes_per_rank("allreduce", 2, S, False) == 4 * S
    # the committed PMC passes agree with the model within 1 % at every N the driver runs
    import json
    pmc = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                      "pmc_traffic.json")))
    for n in (2, 4, 8):
        got = pmc[f"allreduce_f32_256MiB_n{n}"]["bytes_per_launch"]
        assert abs(got / bench.hbm_bytes_per_rank("allreduce", n, S) - 1) < 0.01, (n, got)
        # eager zero-copy (the multi-process default since round 6): 3S - S/n
        got = pmc[f"allreduce_f32_256MiB_n{n}_eager"]["bytes_per_launch"]
        assert abs(got / bench.hbm_bytes_per_rank("allreduce_zero_copy", n, S) - 1) < 0.01, (n, got)
    assert bench.bus_factor("reducescatter", 4) == 0.75 and bench.bus_factor("reduce", 4) == 1.0


def test_size_table_row_from_sweep():
    """The N > 1 suite turns its C4 sweep into an NCCL_AMD_SIZE_TABLE row: LL up to the last size
    where it beats one-shot and direct at every size, then one-shot up to where direct overtakes it."""
    import bench
    K = 1024
    sweep = [{"bytes": b, "ll_us": ll, "oneshot_us": one, "direct_us": d}
             for b, ll, one, d in ((8, 4, 6, 9), (4 * K, 5, 6, 9), (32 * K, 6, 7, 9), (64 * K, 9, 8, 10),
                                   (256 * K, 20, 12, 13), (1 << 20, 60, 30, 25), (4 << 20, 200, 80, 50))]
    row = bench.size_table_row(8, sweep)
    assert (row["ll_bytes"], row["oneshot_bytes"]) == (32 * K, 256 * K)
    assert row["file_line"] == "8 32K - 256K"
    # no one-shot win right after LL: the one-shot range is empty (its limit = LL's)
    sweep[3]["oneshot_us"] = 11   # 64 KiB: LL (9 us) now beats both, so LL extends to 64 KiB
    sweep[4]["oneshot_us"] = 14   # 256 KiB: direct (13 us) beats one-shot
    assert bench.size_table_row(4, sweep)["file_line"] == "4 64K - 64K"
    # LL never wins: 0 turns LL off (one-shot from the first byte, here up to 32 KiB)
    for r in sweep:
        r["ll_us"] = 99
    assert bench.size_table_row(2, sweep)["file_line"] == "2 0 - 32K"
    # a column the sweep did not measure: '-' keeps the built-in value
    for r in sweep:
        del r["ll_us"]
    assert bench.size_table_row(2, sweep)["file_line"] == "2 - - 32K"


def test_scale_decisions_tool_reads_bench_lines():
    """scripts/scale_decisions.py (the round-6 reading of the first 8-GPU SCALE record) finds bench lines wherever
    they sit in a record and calls a difference only outside both columns' spreads."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles", "r05_scale_rehearsal_n8_onegpu.json")
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "scale_decisions.py"), prof],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert "N=8:" in out.stdout and "gather: pull (default) vs push: faster" in out.stdout, out.stdout
    sys.path.insert(0, os.path.join(root, "scripts"))
    import scale_decisions as sd
    line = json.load(open(prof))
    wrapped = {"runs": [{"parsed": {"tail": "noise\n" + json.dumps(line) + "\n"}}]}  # a driver-style record
    assert [d["n_gpus"] for d in sd.bench_lines(wrapped)] == [8]
    a, b = {"ms": 1.0, "ms_min": 0.95, "ms_max": 1.05}, {"ms": 1.08, "ms_min": 1.07, "ms_max": 1.09}
    assert sd.compare(a, b).startswith("within spread")
    b.update(ms=1.2, ms_min=1.19, ms_max=1.21)
    assert sd.compare(a, b).startswith("faster")
