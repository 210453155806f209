"""The C ABI driven from native code: tests/native/nccl_perf (nccl-tests style, built by `make nccl-perf`
against include/nccl.h only) runs AllReduce sum/max over fp32/bf16 (plus ReduceScatter, AllGather and Reduce) with 2 ranks on the one
GPU, eager, hipGraph-replayed and in hold mode, and fails on any wrong element or async error."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "nccl_perf")


@pytest.mark.parametrize("args,forkjoin", [
    (["-b", "8", "-e", "16777216", "-f", "16", "-i", "5"], "0"),
    (["-b", "8", "-e", "1048576", "-f", "32", "-i", "5", "-g", "1"], "0"),
    (["-b", "4", "-e", "4194304", "-f", "64", "-i", "3", "-t", "bf16", "-o", "max"], "0"),
    (["-b", "1024", "-e", "1048576", "-f", "32", "-i", "3"], "1"),
    (["-c", "rs", "-b", "64", "-e", "4194304", "-f", "16", "-i", "5"], "0"),
    (["-c", "ag", "-b", "64", "-e", "4194304", "-f", "16", "-i", "5", "-t", "half"], "0"),
    (["-c", "reduce", "-b", "8", "-e", "4194304", "-f", "16", "-i", "5", "-t", "int", "-o", "max"], "0"),
    (["-b", "8", "-e", "262144", "-f", "8", "-i", "20", "-H", "1"], "0"),
])
def test_native_driver(built, args, forkjoin):
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "nccl-perf"], cwd=ROOT)
    env = dict(os.environ, NCCL_MULTI_RANK_GPU_ENABLE="1", NCCL_AMD_FORK_JOIN=forkjoin,
               NCCL_AMD_SPIN_TIMEOUT_MS="20000")
    out = subprocess.run([EXE, "-r", "2"] + args, env=env, capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stdout + out.stderr
    rows = [l.split() for l in out.stdout.splitlines() if l.strip() and not l.startswith("#")]
    assert rows and all(r[5] == "0" for r in rows), out.stdout  # columns: bytes count time algbw busbw #wrong host


def test_xgmi_probe_loopback(built):
    """The CU-driven peer-bandwidth probe that bench.py's suite runs on multi-GPU nodes, in its one-GPU
    loopback mode: indexing covers every byte of every target (wrong_bytes == 0)."""
    import json
    exe = os.path.join(ROOT, "tests", "native", "xgmi_probe")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "xgmi-probe"], cwd=ROOT)
    out = subprocess.run([exe, "64", "2", "loopback"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert rep["wrong_bytes"] == 0 and rep["write_fanout_GBps"] > 0
    # one rate per link of GPU 0 (the bench line's xgmi_links at N > 1)
    assert len(rep["wt_uncached_write_per_link_GBps"]) == rep["peers"] == len(rep["read_per_link_GBps"])
    assert all(x > 0 for x in rep["wt_uncached_write_per_link_GBps"] + rep["read_per_link_GBps"])
    # the fan-out by workgroup count (the CU budget's per-channel rate)
    assert sorted(int(g) for g in rep["wt_uncached_write_fanout_by_workgroups_GBps"]) == [8, 16, 32, 64, 128, 256]
    assert all(x > 0 for x in rep["wt_uncached_write_fanout_by_workgroups_GBps"].values())


def test_store_atomicity_probe_one_gpu(built):
    """the LL protocol relies on 8-byte single-copy atomicity of the halves of a 16-byte
    write-through store; LL128 would rely on whole 128-byte lines. The probe races a writer (system-scope
    write-through dwordx4 stores into uncached memory, the LL kernels' store) against system-scope 16-byte
    readers on other XCDs of the same GPU. torn8 must be 0; the wider classes are reported (bench.py's
    suite runs the same probe across an xGMI link on multi-GPU nodes)."""
    import json
    exe = os.path.join(ROOT, "tests", "native", "store_atomicity_probe")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "atomicity-probe"], cwd=ROOT)
    out = subprocess.run([exe, "0", "0", "20000", "64", "3000"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    print("store atomicity (one GPU):", rep)
    assert rep["reader_waves"] == 64 and rep["line_observations"] > 0
    assert rep["changed"] > 0, "the readers never raced the writer"
    assert rep["torn8"] == 0, rep


@pytest.mark.parametrize("mode,n", [("pthread", 2), ("pthread", 4), ("initall", 2), ("initall", 4)])
def test_reference_communicator_examples(built, mode, n):
    """The reference's communicator-creation examples as a C program against nccl.h
    (tests/native/comm_examples.cc: docs/examples/01_communicators/02_one_device_per_pthread and
    01_multiple_devices_single_process): per-thread ncclCommInitRank on one unique id, or ncclCommInitAll
    from one thread; rank / count / device queries; a 1M-float AllReduce whose every element must be
    n(n-1)/2; the caller's current device unchanged by every call; Finalize + Destroy. All ranks on the one GPU."""
    exe = os.path.join(ROOT, "tests", "native", "comm_examples")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "comm-examples"], cwd=ROOT)
    env = dict(os.environ, NCCL_MULTI_RANK_GPU_ENABLE="1", NCCL_AMD_SPIN_TIMEOUT_MS="20000")
    out = subprocess.run([exe, mode, str(n)], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr
