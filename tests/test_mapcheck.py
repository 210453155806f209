"""CPU tests of the init-time mapping check (nccl_amd/csrc/mapcheck.cc) with the device and the
imports stubbed (tests/native/mapcheck_test: ranks in host memory, the check kernel emulated, faults injected where
a real mapping could go wrong). A clean set of mappings passes; a mapping that points at other memory, stores that
never arrive, or a hipIpc-fallback mapping that fails make the init return ncclSystemError (2) with one WARN line
per failing (pair, allocation, direction) naming both devices' bus ids and the import path."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "mapcheck_test")


@pytest.fixture(scope="module")
def exe():
    src = os.path.join(ROOT, "tests", "native", "mapcheck_test.cc")
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(src):
        subprocess.check_call(["make", "mapcheck-test"], cwd=ROOT, stdout=subprocess.DEVNULL)
    return EXE


def run(exe, n, *faults):
    env = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    env["NCCL_DEBUG"] = "WARN"
    out = subprocess.run([exe, str(n), *faults], env=env, capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stdout + out.stderr
    res = int(re.search(r"result=(\d+)", out.stdout).group(1))
    warns = [l.split("NCCL WARN ", 1)[1] for l in out.stderr.splitlines() if "NCCL WARN mapping check" in l]
    return res, warns


@pytest.mark.parametrize("n", [2, 3, 8, 16])
def test_clean_mappings_pass(exe, n):
    assert run(exe, n) == (0, [])
    assert run(exe, n, "samepid") == (0, [])


def test_wrong_staging_mapping_names_both_directions(exe):
    res, warns = run(exe, 3, "wrongmap:1:2:0")
    assert res == 2 and len(warns) == 2, warns
    load = [w for w in warns if "<-" in w]
    store = [w for w in warns if "->" in w]
    assert load and "rank 1 (device 1, 0000:11:00.0) <- rank 2 (device 2, 0000:12:00.0)" in load[0]
    assert "staging slab" in load[0] and "dma-buf import" in load[0] and "5a5a5a5a5a5a5a5a" in load[0]
    assert store and "rank 1 (device 1, 0000:11:00.0) -> rank 2 (device 2, 0000:12:00.0)" in store[0]
    assert "did not arrive" in store[0]


def test_flag_block_mapping_and_hipipc_path(exe):
    res, warns = run(exe, 4, "legacy:0:1", "wrongmap:0:1:1")
    assert res == 2
    assert any("<- rank 1" in w and "flag block" in w and "hipIpc handle" in w for w in warns), warns
    assert not any("staging slab" in w for w in warns), warns


def test_dropped_stores_fail_every_peer(exe):
    res, warns = run(exe, 4, "skip:3")
    assert res == 2
    pairs = {(m.group(1), m.group(2)) for w in warns for m in [re.search(r"rank (\d+) \(device.*?-> rank (\d+)", w)] if m}
    assert pairs == {("3", "0"), ("3", "1"), ("3", "2")}, warns
    assert len(warns) == 6  # staging + flags for each of the 3 peers


def test_single_process_peer_pointer_path(exe):
    res, warns = run(exe, 2, "samepid", "wrongmap:0:1:0")
    assert res == 2 and all("hipDeviceEnablePeerAccess" in w for w in warns), warns


def test_second_round_remaps_and_passes(exe):
    """A mapping that fails the first round is re-imported through the export's hipIpc handle (transportRemapPeer,
    stubbed: it repairs the mapping) by the rank that owns it — found from its own loads or from the peer's report of
    its stores — and the second round passes; a mapping the remap cannot repair still fails the init."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    out = subprocess.run([exe, "3", "wrongmap:1:2:0", "fixable:1:2"], env=env, capture_output=True, text=True, timeout=30)
    assert "remap 1<-2" in out.stdout and "result=0" in out.stdout, out.stdout
    out = subprocess.run([exe, "4", "skip:3"], env=env, capture_output=True, text=True, timeout=30)
    assert all(f"remap 3<-{p}" in out.stdout for p in (0, 1, 2)) and "result=2" in out.stdout, out.stdout
    env["NCCL_AMD_MAPCHECK_FALLBACK"] = "0"
    out = subprocess.run([exe, "3", "wrongmap:1:2:0", "fixable:1:2"], env=env, capture_output=True, text=True, timeout=30)
    assert "remap" not in out.stdout and "result=2" in out.stdout, out.stdout


def run_all(exe, n, *args):
    env = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    env["NCCL_DEBUG"] = "WARN"
    out = subprocess.run([exe, str(n), *args], env=env, capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stdout + out.stderr
    return [int(x) for x in re.search(r"results=([\d,]+)", out.stdout).group(1).split(",")], out.stderr


def test_one_thread_per_rank_with_the_bootstrap_exchange(exe):
    """ncclCommInitRank's form: each rank checks its own comm, the barriers and the failure-row all-gather go over the
    (emulated) bootstrap; every rank reaches the same verdict."""
    assert run_all(exe, 4, "threads")[0] == [0, 0, 0, 0]
    res, err = run_all(exe, 4, "threads", "skip:3")
    assert res == [2, 2, 2, 2], err
    res, err = run_all(exe, 3, "threads", "wrongmap:1:2:0", "fixable:1:2")
    assert res == [0, 0, 0], err


def test_a_rank_whose_check_cannot_run_fails_every_rank_at_once(exe):
    """A rank whose part of the check fails (here its kernel launch) still joins the barriers and the all-gather: it
    returns its own error and every peer ncclRemoteError (6) naming it, instead of the peers waiting in a barrier for the
    bootstrap timeout."""
    res, err = run_all(exe, 4, "threads", "runfail:2")
    assert res == [6, 6, 1, 6], err
    assert "rank 2 could not run its part of the check" in err
