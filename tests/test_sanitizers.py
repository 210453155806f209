"""Host sanitizer runs (SURVEY §5 "Race detection"; no GPU): the TCP bootstrap (forked ranks, and ranks as
threads of one process as ncclCommInitAll runs them), the IPC fd server (concurrent fetches, publish / retire
churn, bounded failures, stop under load) and the planning code, built with ASan+UBSan and, separately, TSan
(Makefile target `sanitize`; host code only, nothing on the GPU is instrumented). A run passes when it exits 0
and no sanitizer printed a report."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPORTS = ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:", "WARNING: ThreadSanitizer")


@pytest.fixture(scope="module")
def sanitized():
    r = subprocess.run(["make", "-j8", "sanitize"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return os.path.join(ROOT, "build")


def _run(path, *args, **env):
    e = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    e.update(NCCL_AMD_BOOTSTRAP_TIMEOUT_MS="20000", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
             LSAN_OPTIONS="suppressions=" + os.path.join(ROOT, "tests", "native", "lsan.supp"),
             TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1", UBSAN_OPTIONS="print_stacktrace=1")
    e.update({k: str(v) for k, v in env.items()})
    r = subprocess.run([path, *args], env=e, capture_output=True, text=True, timeout=180)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert not any(s in out for s in REPORTS), out[-4000:]
    return out


@pytest.mark.parametrize("san,args", [("asan", ("5", "4")), ("asan", ("5", "4", "threads")),
                                      ("tsan", ("6", "4", "threads")), ("asan", ("5", "2", "scalable", "3"))])
def test_bootstrap_sanitized(sanitized, san, args):
    out = _run(os.path.join(sanitized, san, "bootstrap_test"), *args)
    assert "failures=0" in out and "roots_left=0" in out if "scalable" in args else "failures=0" in out


@pytest.mark.parametrize("san,args", [("asan", ()), ("tsan", ("nofork",))])
def test_ipc_fd_server_sanitized(sanitized, san, args):
    assert "failures=0" in _run(os.path.join(sanitized, san, "ipc_server_test"), *args)


def test_planning_asan(sanitized):
    exe = os.path.join(sanitized, "asan", "plan_test")
    for n, f, dt, count in ((1, "ar", 7, 1000), (2, "ar", 7, 3), (8, "ar", 9, 1 << 26), (8, "rs", 6, 1 << 20),
                            (8, "ag", 0, 4097), (8, "reduce", 2, 1 << 25), (3, "reduce", 4, 777)):
        assert "algo=" in _run(exe, str(n), f, str(dt), str(count))
    _run(exe, "4", "ar", "7", str(1 << 22), NCCL_ALGO="TREE")
    # the ring AllReduce's reference partition (enqueue.cc ringParts): one channel, many channels, tiny chunks
    for n, dt, count, cap in ((2, 7, 1 << 26, 256), (3, 8, 100_003, 7), (8, 10, 5, 1), (4, 6, (1 << 30) + 3, 64)):
        assert "algo=ring" in _run(exe, str(n), "ar", str(dt), str(count), "0", str(cap), NCCL_ALGO="RING",
                                   NCCL_BUFFSIZE="16384")
    out = _run(exe, "2", "batch", *[f"rs:9:{2 * c}" for c in (100, 2000, 100_000, 1_000_000)], "ag:7:5000",
               *(["ar:7:100000"] * 10))
    assert out.count("algo=") == 5
