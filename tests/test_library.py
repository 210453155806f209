"""CPU tests of the product library's host side: the C ABI loads and exports every symbol that
include/nccl.h declares, version / error strings / argument checks behave like the reference, and
the TCP bootstrap works across processes. No compute call is made (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import nccl_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "nccl.h")).read()
    return sorted(set(re.findall(r"^\s*(?:ncclResult_t|const char\*)\s+(p?nccl\w+)\s*\(", src, re.M)))


def test_exports_every_declared_symbol(built):
    lib = nccl_amd.load()
    names = _declared_functions()
    assert len(names) >= 48
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the python mirror binds exactly the non-profiling set
    assert sorted(nccl_amd.EXPORTED) == sorted(n for n in names if not n.startswith("p"))


def test_exports_are_nccl_only(built):
    """Every defined dynamic symbol of any kind (T, V, W, B, D, ...) is a declared nccl* / pnccl* function: the
    reference's export surface (src/libnccl.map:13-19, `local: *`), enforced by nccl_amd/csrc/libnccl.map."""
    out = subprocess.check_output(["nm", "-D", "--defined-only", nccl_amd.LIB_PATH], text=True)
    syms = [l.split()[-1] for l in out.splitlines() if l.strip()]
    syms = [s.split("@")[0] for s in syms]
    assert sorted(syms) == _declared_functions(), sorted(set(syms) ^ set(_declared_functions()))[:20]


def test_version_and_error_strings(built):
    assert nccl_amd.get_version() == 23007  # NCCL_VERSION(2,30,7), nccl.h.in:26
    lib = nccl_amd.load()
    assert lib.ncclGetErrorString(0) == b"no error"
    assert lib.ncclGetErrorString(4).startswith(b"invalid argument")
    assert lib.ncclGetErrorString(5).startswith(b"invalid usage")
    assert lib.ncclGetErrorString(7) == b"NCCL operation in progress"
    assert lib.ncclGetErrorString(99) == b"unknown result code"


def test_unique_id_is_128_bytes_and_distinct(built):
    a, b = nccl_amd.get_unique_id(), nccl_amd.get_unique_id()
    assert len(a) == 128 and len(b) == 128 and a != b


def test_argument_checks_without_gpu(built):
    lib = nccl_amd.load()
    P = ctypes.c_void_p
    # invalid comm (NULL) -> ncclInvalidArgument (argcheck.cc:30-45)
    assert lib.ncclAllReduce(None, None, 10, 7, 0, None, None) == 4
    assert lib.ncclReduce(None, None, 10, 7, 0, 0, None, None) == 4
    # bad rank count / rank (init.cc: ncclCommInitRankDev checks) before any device call
    c = P()
    uid = nccl_amd._uid(nccl_amd.get_unique_id())
    assert lib.ncclCommInitRank(ctypes.byref(c), 0, uid, 0) == 4
    assert lib.ncclCommInitRank(ctypes.byref(c), 2, uid, 2) == 4
    assert lib.ncclCommInitRank(ctypes.byref(c), 2, uid, -1) == 4
    # bad config magic
    cfg = nccl_amd.Config.default()
    cfg.magic = 0
    assert lib.ncclCommInitRankConfig(ctypes.byref(c), 2, uid, 0, ctypes.byref(cfg)) == 4
    # unmatched group end -> ncclInvalidUsage
    assert lib.ncclGroupEnd() == 5
    assert lib.ncclGroupStart() == 0 and lib.ncclGroupEnd() == 0
    # an invalid call inside a group poisons the group (reference group.cc error propagation)
    assert lib.ncclGroupStart() == 0
    assert lib.ncclAllReduce(None, None, 10, 7, 0, None, None) == 4
    assert lib.ncclGroupEnd() == 4
    v = ctypes.c_int()
    assert lib.ncclCommCount(None, ctypes.byref(v)) == 4
    assert lib.ncclGetVersion(None) == 4
    # destroying / aborting NULL is a no-op
    assert lib.ncclCommDestroy(None) == 0 and lib.ncclCommAbort(None) == 0
    assert b"NULL" in lib.ncclGetLastError(None) or lib.ncclGetLastError(None) != b""


@pytest.mark.parametrize("n", [2, 5, 8])
def test_bootstrap_across_processes(built, n):
    exe = os.path.join(ROOT, "build", "bootstrap_test")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "bootstrap-test"], cwd=ROOT)
    env = dict(os.environ, NCCL_AMD_BOOTSTRAP_TIMEOUT_MS="20000")
    r = subprocess.run([exe, str(n), "4"], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("n,nid", [(4, 2), (5, 3), (2, 5), (8, 8)])
def test_bootstrap_scalable_ids(built, n, nid):
    """ncclCommInitRankScalable's rendezvous (reference init.cc:2695-2728): the ranks meet at id 0, the
    other ids' roots are released by exactly one rank each (the reference's rank-to-root partition,
    bootstrap.cc:59-69) and stop listening; nid > n included."""
    subprocess.check_call(["make", "-s", "bootstrap-test"], cwd=ROOT)
    exe = os.path.join(ROOT, "build", "bootstrap_test")
    env = dict(os.environ, NCCL_AMD_BOOTSTRAP_TIMEOUT_MS="20000")
    r = subprocess.run([exe, str(n), "2", "scalable", str(nid)], env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0 and "roots_left=0" in r.stdout, r.stdout + r.stderr


def test_new_api_argument_checks_without_gpu(built):
    """ncclCommInitRankScalable / ncclCommMemStats / ncclGroupSimulateEnd argument checks (no GPU)."""
    lib = nccl_amd.load()
    P = ctypes.c_void_p
    c = P()
    assert lib.ncclCommInitRankScalable(ctypes.byref(c), 2, 0, 0, None, None) == 4   # nId < 1
    v = ctypes.c_uint64()
    assert lib.ncclCommMemStats(None, 3, ctypes.byref(v)) == 4                      # NULL comm
    si = nccl_amd.SimInfo.default()
    assert lib.ncclGroupSimulateEnd(ctypes.byref(si)) == 5                          # not in a group
    bad = nccl_amd.SimInfo.default()
    bad.magic = 0
    assert lib.ncclGroupStart() == 0
    assert lib.ncclGroupSimulateEnd(ctypes.byref(bad)) == 4                         # uninitialised struct
    assert lib.ncclGroupStart() == 0                                                # empty group: 0 us
    assert lib.ncclGroupSimulateEnd(ctypes.byref(si)) == 0 and si.estimatedTime == 0.0


def test_registration_argument_checks_without_gpu(built):
    lib = nccl_amd.load()
    P = ctypes.c_void_p
    h = P()
    assert lib.ncclCommRegister(None, P(16), 64, ctypes.byref(h)) == 4       # NULL comm
    assert lib.ncclCommDeregister(None, None) == 4
    w = P()
    assert lib.ncclCommWindowRegister(None, P(16), 64, ctypes.byref(w), 1) == 4
    assert lib.ncclCommWindowDeregister(None, None) == 4
    out = P()
    assert lib.ncclWinGetUserPtr(None, None, ctypes.byref(out)) == 4


def test_tuner_plugin_abi_mock(built):
    """Drive the test tuner plugin through the v6 struct exactly as libnccl.so does (reference
    plugins/tuner/example/test/test_plugin.c style: no GPU, synthetic sizes)."""
    path = os.path.join(ROOT, "tests", "native", "libnccl-tuner-test.so")
    if not os.path.exists(path):
        subprocess.check_call(["make", "tuner-test"], cwd=ROOT)
    lib = ctypes.CDLL(path)
    P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    INIT = ctypes.CFUNCTYPE(I, ctypes.POINTER(P), ctypes.c_uint64, S, S, P, P, P)
    GET = ctypes.CFUNCTYPE(I, P, I, S, I, P, I, I, I, ctypes.POINTER(I))
    FIN = ctypes.CFUNCTYPE(I, P)

    class V6(ctypes.Structure):
        _fields_ = [("name", ctypes.c_char_p), ("init", INIT), ("getCollInfo", GET), ("finalize", FIN),
                    ("getChunkSize", P)]

    t = V6.in_dll(lib, "ncclTunerPlugin_v6")
    assert t.name == b"mi355x-test"
    ctx = P()
    assert t.init(ctypes.byref(ctx), 1, 8, 1, None, None, None) == 0
    table = (ctypes.c_float * 21)(*([-1.0] * 21))      # [7 algorithms][3 protocols]
    table[1 * 3 + 2] = 12.5                             # RING/SIMPLE offered
    table[0 * 3 + 2] = 9.0                              # TREE/SIMPLE offered
    nch = I(0)
    os.environ["TEST_TUNER_FORCE"] = "ring_simple"
    os.environ["TEST_TUNER_NCH"] = "5"
    try:
        assert t.getCollInfo(ctx, 4, 1 << 20, 1, ctypes.cast(table, P), 7, 3, 0, ctypes.byref(nch)) == 0
    finally:
        os.environ.pop("TEST_TUNER_FORCE")
        os.environ.pop("TEST_TUNER_NCH")
    assert table[1 * 3 + 2] == 0.0 and table[0 * 3 + 2] == 9.0 and nch.value == 5
    assert table[0] == -1.0                             # ignored entries stay ignored
    assert lib.testTunerCalls() == 1 and lib.testTunerLastFunc() == 4
    assert t.finalize(ctx) == 0
