"""bench.py's N>1 harness end to end on the one-GPU box: torchrun with 2 ranks (each a process on the same
GPU), quick suite. Guards the unique-id exchange, barriers, max-over-ranks timing, the suite's extra
communicators and windows, and the one JSON line the driver parses — the code the round-end multi-GPU
run executes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_quick(built):
    env = dict(os.environ, NCCL_AMD_SPIN_TIMEOUT_MS="20000")
    env.pop("NCCL_AMD_EAGER_REGISTER", None)  # the library's defaults, as the driver runs it
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--quick-suite", "--cpu-seconds", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["check"] == "pass" and d["value"] > 0 and d["unit"] == "GB/s"
    # value = the metric's busBW (per rank); the whole-job sum is reported beside it
    assert d["value"] == d["busbw_GBps"] and abs(d["busbw_sum_GBps"] - 2 * d["busbw_GBps"]) < 0.05
    # at n >= 2 the binding roofline is the links; the HBM fraction is secondary, and the
    # kernel is named from the run (the library's kernel log), not a literal
    roof = d["roofline"]
    assert roof["bound"] == "xgmi" and roof["unit"] == "GB/s" and roof["peak"] > 0, roof
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    assert 0.5 < roof["achieved"] / d["busbw_GBps"] < 2.0   # per-launch event time vs the whole step's wall time
    assert "hbm" in roof and roof["hbm"]["peak"] == 8000.0
    # the library's defaults: the staged direct kernel, its HBM model (3S + 2(n-1)/n S = 4S at n = 2)
    assert roof["kernel"] and "ncclamd::collKernel<float, 0, 0>" in roof["kernel"], roof["kernel"]
    assert "direct scatter-reduce-gather" in d["config"]["workload"], d["config"]
    assert roof["hbm"]["algorithmic_bytes_per_launch"] == 4 * 256 * 2**20, roof["hbm"]
    # every N line carries the host-core baseline (rank 0, same run) and the PMC traffic
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1, d["cpu_baseline"]
    assert roof["traffic"] and roof["traffic"] > 0, roof
    s = d["suite"]
    assert "error" not in s, s
    assert s["rs_ag_bf16"]["check"] == "pass" and s["reduce_int32"]["check"].startswith("pass")
    assert s["symmetric_window"]["check"].startswith("pass")
    assert s["registered"]["check"].startswith("pass")
    assert all(r["check"].startswith("pass") for r in s["staged_tuning"]["runs"]), s["staged_tuning"]
    # every column timed in >= 3 interleaved rounds, median with its spread
    assert all(r["reps"] >= 3 and r["ms_min"] <= r["ms"] <= r["ms_max"] for r in s["staged_tuning"]["runs"])
    # the unregistered headline buffers registered on first use, bitwise = the staged result
    assert s["eager_zero_copy"]["check"].startswith("pass") and s["eager_zero_copy"]["ms"] > 0, s["eager_zero_copy"]
    assert s["group_aggregation"]["aggregated_us_per_group"] > 0 and s["group_aggregation"]["check"].startswith("pass")
    assert s["symmetric_window"]["ar_fp16_sweep_check"].startswith("pass")
    # every column of the C4 sweep checked at every size (exact integer sums)
    assert all(v.startswith("pass") for v in s["ar_fp16_sweep_check"].values()), s["ar_fp16_sweep_check"]
    # the C4 sweep's crossovers as a ready NCCL_AMD_SIZE_TABLE row
    assert s["size_table_row"]["file_line"].startswith("2 "), s["size_table_row"]
    # the link probe and the fence on / off column at the top level of the N > 1 line
    assert "xgmi_links" in d and d["p2p_fence"]["check"] == "pass", (d.get("xgmi_links"), d.get("p2p_fence"))
    assert d["p2p_fence"]["fence_on_ms"] > 0 and d["p2p_fence"]["fence_off_ms"] > 0


def test_bench_one_gpu_line(built):
    """The N=1 line (a short run): HBM roofline of the one-rank copy kernel, named from the run, with the
    cold-buffer fraction beside the headline one."""
    env = dict(os.environ, NCCL_AMD_SPIN_TIMEOUT_MS="20000")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2", "--cpu-seconds", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    d = json.loads(lines[-1])
    roof = d["roofline"]
    assert d["n_gpus"] == 1 and d["check"] == "pass" and roof["bound"] == "hbm"
    assert "copyKernel" in roof["kernel"], roof
    assert 0 < roof["frac_cold"] <= 1.0 and roof["achieved_cold"] > 0
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] >= 1
    # the host-staged bucket: the pipelined copies and the collective on the pinned host buffers, both bitwise equal
    # to the one-stream result
    hs = d["host_staged"]
    assert hs["pipelined"]["check"] == "pass" and hs["direct"]["check"] == "pass", hs
    assert hs["direct"]["ms_per_step"] > 0


def test_bench_reports_a_failed_init(built):
    """A communicator init that fails on every rank (here the mapping check with every rank's stores dropped, as a
    broken cross-device mapping would) still gives the driver its one JSON line: value 0, check FAIL and the
    library's error, and a non-zero exit — not a run that ends without output."""
    env = dict(os.environ, NCCL_AMD_SPIN_TIMEOUT_MS="20000", NCCL_AMD_MAPCHECK_FAULT="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--quick-suite", "--no-cpu-baseline"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert out.returncode != 0
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:] + out.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["value"] == 0.0 and d["check"] == "FAIL" and "init failed" in d["error"], d
    assert "mapping check" in d["error"] and "did not arrive" in d["error"], d
    assert "NCCL WARN mapping check" in out.stderr, out.stderr[-3000:]  # bench.py turns on NCCL_DEBUG=WARN
