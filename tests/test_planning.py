"""CPU tests of the host-side planning in enqueue.cc (no GPU): tests/native/plan_test compiles enqueue.cc
with the launches and the few HIP calls stubbed and prints the plan of one collective. Checks the size
table (LL / one-shot / direct crossovers and how they scale with n), NCCL_ALGO / NCCL_PROTO (reference
syntax), the LL alignment and capacity rules, the co-residency channel cap, the ReduceScatter / AllGather LL
range, the rootless Reduce block split, and the invariants every plan must satisfy for the kernels' indexing to be in bounds."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "plan_test")
SIZES = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2, 10: 1, 11: 1}


@pytest.fixture(scope="module")
def exe():
    src = os.path.join(ROOT, "tests", "native", "plan_test.cc")
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(src):
        subprocess.check_call(["make", "plan-test"], cwd=ROOT, stdout=subprocess.DEVNULL)
    return EXE


def plan(exe, n, func, dtype, count, offset=0, chancap=256, **env):
    e = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    e.update({k: str(v) for k, v in env.items()})
    out = subprocess.run([exe, str(n), func, str(dtype), str(count), str(offset), str(chancap)], env=e,
                         capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stdout + out.stderr
    return {k: (v if k == "algo" else int(v)) for k, v in (t.split("=") for t in out.stdout.split())}


@pytest.mark.parametrize("n,nbytes,algo", [
    (1, 4096, "copy"), (1, 256 << 20, "copy"),
    (2, 8, "ll"), (2, 64 << 10, "ll"), (2, 128 << 10, "ll"), (2, 256 << 10, "oneshot"), (2, 1 << 20, "oneshot"), (2, 2 << 20, "oneshot"),
    (2, 4 << 20, "direct"), (2, 256 << 20, "direct"),
    (4, 64 << 10, "ll"), (4, 128 << 10, "oneshot"), (4, 512 << 10, "oneshot"), (4, 1 << 20, "direct"),
    (8, 16 << 10, "ll"), (8, 32 << 10, "ll"), (8, 64 << 10, "oneshot"), (8, 256 << 10, "oneshot"),
    (8, 512 << 10, "direct"), (8, 256 << 20, "direct"),
])
def test_allreduce_size_table(exe, n, nbytes, algo):
    assert plan(exe, n, "ar", 7, nbytes // 4)["algo"] == algo


def test_proto_and_algo_overrides(exe):
    assert plan(exe, 8, "ar", 7, (256 << 10) // 4, NCCL_PROTO="LL")["algo"] == "ll"        # LL to capacity
    assert plan(exe, 2, "ar", 7, 1024, NCCL_PROTO="^LL")["algo"] == "oneshot"
    assert plan(exe, 2, "ar", 7, 1024, NCCL_PROTO="Simple")["algo"] == "oneshot"
    assert plan(exe, 2, "ar", 7, 1024, NCCL_PROTO="LL,Simple")["algo"] == "ll"
    assert plan(exe, 2, "ar", 7, 1024, NCCL_ALGO="DIRECT")["algo"] == "direct"
    assert plan(exe, 2, "ar", 7, 1024, NCCL_ALGO="RING")["algo"] == "ring"
    assert plan(exe, 8, "ar", 7, 64 << 20, NCCL_ALGO="ONESHOT")["algo"] == "oneshot"
    assert plan(exe, 2, "ar", 7, 1024, NCCL_ALGO="DIRECT", NCCL_PROTO="LL")["algo"] == "ll"  # only LL left
    assert plan(exe, 2, "ar", 7, 100_000, NCCL_AMD_LL_BYTES=1 << 20)["algo"] == "ll"
    assert plan(exe, 2, "ar", 7, 4_000_000, NCCL_AMD_ONESHOT_BYTES=64 << 20)["algo"] == "oneshot"


def matrix(exe, **env):
    """loadTuning's per-collective resolution of NCCL_ALGO / NCCL_PROTO (plan_test matrix)."""
    e = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    e.update({k: str(v) for k, v in env.items()})
    out = subprocess.run([exe, "matrix"], env=e, capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = out.stdout.split("\n")
    res = {"parse": int(lines[0].split("=")[1])}
    for line in lines[1:]:
        if line:
            d = dict(t.split("=") for t in line.split())
            func = d.pop("func")
            res[func] = {k: (v if k == "algo" else int(v)) for k, v in d.items()}
    return res


def protos(row):
    return {p for p in ("ll", "ll128", "simple") if row[p]}


def test_proto_grammar_reference_examples(exe):
    """NCCL_PROTO / NCCL_ALGO follow the reference's parseList grammar (src/graph/tuning.cc:36-136):
    comma lists, '^' exclusion, 'func:list' entries separated by ';', case-insensitive names. The three examples of
    tuning.cc:43-54 / env.rst:1304-1310."""
    m = matrix(exe, NCCL_PROTO="LL,Simple;allreduce:^LL")   # LL + Simple everywhere, all but LL for AllReduce
    assert m["parse"] == 0
    assert protos(m["allreduce"]) == {"simple"}               # (LL128 stays at the engine's gate, off)
    for f in ("reducescatter", "allgather", "reduce"):
        assert protos(m[f]) == {"ll", "simple"}, f
    m = matrix(exe, NCCL_PROTO="^LL128;allreduce:LL128")     # everything but LL128, only LL128 for AllReduce
    assert protos(m["allreduce"]) == {"ll128"}
    assert protos(m["reducescatter"]) == {"ll", "simple"}
    m = matrix(exe, NCCL_ALGO="ring,collnetdirect;allreduce:tree,collnetdirect;broadcast:ring")
    assert m["parse"] == 0
    assert m["allreduce"]["algo"] == "tree"                   # Tree (+ CollNetDirect, absent here)
    for f in ("reducescatter", "allgather", "reduce"):
        assert m[f]["algo"] == "ring", f
    # the list forms the old single-name parser got wrong
    m = matrix(exe, NCCL_ALGO="Ring,Tree")                    # several: the size table over one-shot and direct
    assert all(m[f]["algo"] == "none" and m[f]["oneshot"] and m[f]["direct"] and not m[f]["noalgo"]
               for f in ("allreduce", "reducescatter", "allgather", "reduce"))
    m = matrix(exe, NCCL_ALGO="^Tree")                        # Ring + the rest: still several implemented
    assert m["allreduce"]["algo"] == "none" and m["allreduce"]["oneshot"] and m["allreduce"]["direct"]
    m = matrix(exe, NCCL_ALGO="^Tree,OneShot,Direct")         # only Ring left of the implemented ones
    assert m["allreduce"]["algo"] == "ring"
    m = matrix(exe, NCCL_ALGO="Ring,Direct")                  # RING/SIMPLE stands for direct: no one-shot
    assert m["allreduce"]["algo"] == "none" and not m["allreduce"]["oneshot"] and m["allreduce"]["direct"]
    m = matrix(exe, NCCL_ALGO="tree,ONESHOT", NCCL_PROTO="ll,SIMPLE")   # case-insensitive
    assert m["parse"] == 0 and m["allreduce"]["oneshot"] and not m["allreduce"]["direct"]
    m = matrix(exe, NCCL_PROTO="^LL,Simple")                  # LL128 the only protocol left: on
    assert protos(m["allreduce"]) == {"ll128"}
    m = matrix(exe, NCCL_PROTO="^LL")                         # LL128 at its gate (NCCL_AMD_LL128)
    assert protos(m["allreduce"]) == {"simple"}
    assert protos(matrix(exe, NCCL_PROTO="^LL", NCCL_AMD_LL128=1)["allreduce"]) == {"ll128", "simple"}


@pytest.mark.parametrize("var,val", [
    ("NCCL_PROTO", "Foo"), ("NCCL_PROTO", "LL,Simple;LL128"),      # unknown name; a later entry without prefix
    ("NCCL_PROTO", "bogus:LL"), ("NCCL_ALGO", "Ring;allreduce:Spiral"), ("NCCL_ALGO", "Ring,Tre"),
    ("NCCL_ALGO", "allreduce:"),                                   # 'allreduce' read as a name, as strtok does
])
def test_proto_grammar_errors(exe, var, val):
    """An unknown token or prefix is ncclInvalidUsage (reference tuning.cc:73-75, 108-121); init fails on every rank
    (CommTuning::parseError, agreed at init; GPU: test_gpu_api.py test_init_fails_on_bad_algo_proto)."""
    assert matrix(exe, **{var: val})["parse"] == 5


def test_per_function_enables_drive_the_plan(exe):
    # AllReduce Simple only, ReduceScatter LL + Simple (the reference's own example)
    env = dict(NCCL_PROTO="LL,Simple;allreduce:^LL")
    assert plan(exe, 2, "ar", 7, 1000, **env)["algo"] == "oneshot"
    assert plan(exe, 2, "rs", 7, 1000, **env)["algo"] == "ll"
    assert plan(exe, 2, "ar", 7, 1000)["algo"] == "ll"
    # per-function algorithms: AllReduce on the chain, ReduceScatter on the ring
    env = dict(NCCL_ALGO="ring;allreduce:tree")
    assert plan(exe, 4, "ar", 7, 1 << 20, **env)["algo"] == "chain"
    assert plan(exe, 4, "rs", 7, 1 << 20, **env)["algo"] == "ring"
    # several algorithms: the size table; 'Ring,Direct' has no one-shot stand-in -> direct where one-shot would run
    assert plan(exe, 2, "ar", 7, 100_000, NCCL_ALGO="Ring,Tree")["algo"] == "oneshot"
    assert plan(exe, 2, "ar", 7, 100_000, NCCL_ALGO="Ring,Direct")["algo"] == "direct"
    assert plan(exe, 2, "ar", 7, 1000, NCCL_ALGO="Ring,Direct")["algo"] == "ll"
    assert plan(exe, 2, "ar", 7, 64 << 20, NCCL_ALGO="Tree,OneShot")["algo"] == "oneshot"  # no direct stand-in
    # only algorithms absent from an xGMI mesh, or no protocol: the collective fails with ncclInvalidUsage
    # (reference enqueue.cc:2052-2065), the other collectives still plan
    for env in (dict(NCCL_ALGO="NVLS"), dict(NCCL_ALGO="allreduce:PAT,CollNetChain"),
                dict(NCCL_PROTO="allreduce:^LL,LL128,Simple")):
        out = subprocess.run([exe, "2", "ar", "7", "1000"], env={**{k: v for k, v in os.environ.items()
                                                                  if not k.startswith("NCCL_")}, **env},
                             capture_output=True, text=True, timeout=30)
        assert out.returncode == 1 and "error=5" in out.stdout, (env, out.stdout)
    assert plan(exe, 2, "rs", 7, 1000, NCCL_ALGO="allreduce:PAT")["algo"] == "ll"


def test_ll_choice_is_rank_uniform_and_needs_room(exe):
    # the protocol must not depend on this rank's buffer alignment (peers may be aligned differently):
    # misaligned buffers take LL too and the kernel handles any alignment (enqueue.cc:205)
    for off in (1, 2, 4, 8):
        assert plan(exe, 2, "ar", 7, 1001, offset=off)["algo"] == "ll"
    assert plan(exe, 8, "reduce", 7, 1001, offset=4)["algo"] == "ll"
    big = plan(exe, 2, "ar", 7, (512 << 10) // 4, NCCL_PROTO="LL")        # exactly the line area
    assert big["algo"] == "ll" and big["part"] * 16 <= 32 << 10
    assert plan(exe, 2, "ar", 7, (1 << 20) // 4, NCCL_PROTO="LL,Simple", NCCL_AMD_LL_BYTES=4 << 20)["algo"] == "oneshot"


def test_reduce_size_table(exe):
    # LL (lines to every peer, the root folds) up to the AllReduce LL limit, direct above; no one-shot
    assert plan(exe, 8, "reduce", 9, 1)["algo"] == "ll"
    assert plan(exe, 8, "reduce", 9, 1000)["algo"] == "ll"
    assert plan(exe, 2, "reduce", 7, (128 << 10) // 4)["algo"] == "ll"
    assert plan(exe, 2, "reduce", 7, (128 << 10) // 4 + 1)["algo"] == "direct"
    assert plan(exe, 8, "reduce", 9, 1 << 20)["algo"] == "direct"
    assert plan(exe, 8, "reduce", 9, 1000, NCCL_PROTO="^LL")["algo"] == "direct"


@pytest.mark.parametrize("func", ["rs", "ag"])
def test_blocked_collectives_size_table(exe, func):
    # LL while a rank block is within 256 KiB / n (256 KiB of total data), direct above; the blocks
    # must be 8-byte aligned (count * sizeof(T) % 8 == 0) for the line payloads
    for n in (2, 4, 8):
        limit = (256 << 10) // n // 4          # fp32 elements per block at the limit
        assert plan(exe, n, func, 7, 2)["algo"] == "ll"
        assert plan(exe, n, func, 7, limit)["algo"] == "ll"
        assert plan(exe, n, func, 7, limit + 2)["algo"] == "direct"
        assert plan(exe, n, func, 7, 1)["algo"] == "direct"   # 4-byte blocks: no LL
        assert plan(exe, n, func, 8, 1)["algo"] == "ll"       # one fp64 per block
    assert plan(exe, 2, func, 7, 1000, NCCL_PROTO="^LL")["algo"] == "direct"
    assert plan(exe, 2, func, 7, 1000, offset=4)["algo"] == "ll"   # alignment is rank-local: never decides
    p = plan(exe, 8, func, 7, 1000)
    assert p["chunk"] == 1000 and p["part"] * p["nch"] * 8 >= 4000


def test_rootless_reduce_blocks(exe):
    # n >= 3: n-1 blocks (root owns none), each alignUp(divUp(count, n-1), 16/sizeof(T)) elements
    for n, count in ((3, 1), (4, 999_999), (8, 33_554_432)):
        p = plan(exe, n, "reduce", 2, count, NCCL_PROTO="^LL")
        epp = 16 // 4
        want = -(-count // (n - 1))
        want = -(-want // epp) * epp
        assert p["chunk"] == want, (n, count, p)
    p = plan(exe, 2, "reduce", 2, 1000, NCCL_PROTO="^LL")  # n = 2 keeps one block per rank
    assert p["chunk"] == 500


@pytest.mark.parametrize("n,func,dtype,count", [
    (2, "ar", 7, 67_108_864), (8, "ar", 7, 67_108_864), (8, "ar", 6, 12_345_679), (3, "ar", 8, 7_777_777),
    (8, "rs", 9, 67_108_864), (8, "ag", 9, 67_108_864), (8, "reduce", 2, 33_554_432), (5, "ar", 0, 3_000_001),
])
def test_plan_invariants(exe, n, func, dtype, count):
    p = plan(exe, n, func, dtype, count)
    ts = SIZES[dtype]
    epp = 16 // ts
    assert p["algo"] == "direct"
    assert 1 <= p["nch"] <= 256
    assert p["part"] % epp == 0 and p["slice"] % epp == 0 and 0 < p["slice"] <= p["part"]
    assert p["steps"] == -(-p["part"] // p["slice"])
    assert p["part"] * p["nch"] >= p["chunk"]          # the channels cover a whole rank block
    if func == "ar":
        assert p["chunk"] * n >= count and p["chunk"] % epp == 0
    if func in ("rs", "ag"):
        assert p["chunk"] == count


def test_channel_cap(exe):
    # several ranks per GPU: every channel of a launch must be co-resident, so plans respect chanCap — every
    # algorithm, the reference-partition ones with any NCCL_AMD_REF_NCHANNELS included (the launch guard,
    # enqueue.cc checkGrid, refuses a plan past the cap rather than index past the staging)
    for cap in (1, 3, 7, 64):
        assert plan(exe, 4, "ar", 7, 64 << 20, chancap=cap)["nch"] <= cap
        assert plan(exe, 4, "ar", 7, 1000, chancap=cap, NCCL_PROTO="LL")["nch"] <= cap
        for env in ({"NCCL_ALGO": "RING"}, {"NCCL_AMD_REF_ORDER": 1}, {"NCCL_ALGO": "TREE"}):
            for k in (1, 5, 64, 100):
                for count in (1000, 100_003, 1 << 22):
                    p = plan(exe, 3, "ar", 7, count, chancap=cap, NCCL_AMD_REF_NCHANNELS=k,
                             NCCL_AMD_MIN_CHANNEL_BYTES=1024, **env)
                    assert 1 <= p["nch"] <= cap, (cap, env, k, count, p)


@pytest.mark.parametrize("rpg", [1, 2, 3, 4, 5, 8, 16])
def test_co_resident_channel_cap_leaves_half_the_slots_free(exe, rpg):
    """ranks sharing a GPU get CUs / ranks-per-GPU channels per launch, half of the 2 x CUs slots
    kept free (enqueue.cc coResidentChannelCap): round 5's n = 8 rehearsal stalled once at 8 ranks x 64 = 512 = every
    slot, for a cause not established. One rank per GPU keeps 2 x CUs."""
    for cus in (256, 304, 80, 7):
        cap = int(subprocess.run([exe, "cap", str(cus), str(rpg)], capture_output=True, text=True,
                                 timeout=30).stdout)
        slots = 2 * cus
        if rpg == 1:
            assert cap == slots
        else:
            assert cap >= 1 and (2 * rpg * cap <= slots or cap == 1), (cus, rpg, cap)   # half the slots at most
            assert 2 * rpg * (cap + 1) > slots or cap == 1                # and no more is given away
    # MI355X: 256 CUs -> 128 / 64 / 32 channels per rank at 2 / 4 / 8 ranks per GPU (round 5: 256 / 128 / 64)
    assert [int(subprocess.run([exe, "cap", "256", str(r)], capture_output=True, text=True).stdout)
            for r in (2, 4, 8)] == [128, 64, 32]


def test_ll_channels_never_empty(exe):
    # every LL channel of an op carries >= 1 payload: an empty channel would advance its epoch without
    # exchanging lines and break the parity double-buffering (enqueue.cc:224)
    for count, env in ((80, {"NCCL_AMD_LL_CHANNEL_BYTES": 8}), (7, {"NCCL_AMD_LL_CHANNEL_BYTES": 8}),
                       (1000, {}), (33, {"NCCL_AMD_LL_CHANNEL_BYTES": 16})):
        p = plan(exe, 2, "ar", 7, count, **env)
        npk = -(-count * 4 // 8)
        assert p["algo"] == "ll"
        assert p["nch"] * p["part"] >= npk and (p["nch"] - 1) * p["part"] < npk, (count, env, p)


@pytest.mark.parametrize("func,algo,want", [
    ("ar", "RING", ("ring", 0)), ("rs", "RING", ("ring", 1)), ("ag", "RING", ("ring", 2)),
    ("ar", "TREE", ("chain", 3)), ("reduce", "RING", ("chain", 4)),
    ("rs", "TREE", ("direct", None)), ("ag", "TREE", ("direct", None)), ("reduce", "TREE", ("direct", None)),
])
def test_forced_reference_algorithms(exe, func, algo, want):
    # NCCL_ALGO=RING / TREE run the reference's own algorithms (pipe.h); where the reference has none
    # (TREE for RS / AG / Reduce) the default plan runs, with a warning
    for n, count in ((2, 1000), (8, 1 << 20), (3, 7)):
        p = plan(exe, n, func, 7, count * (n if func == "rs" else 1), NCCL_ALGO=algo)
        assert p["algo"] == want[0], (n, count, p)
        if want[1] is not None:
            assert p["kind"] == want[1]
            if want[1] != 0:  # (the ring AllReduce's partition: test_ring_allreduce_takes_the_reference_partition)
                assert p["part"] * p["nch"] >= p["chunk"] and p["steps"] == -(-p["part"] // p["slice"])
            if want[0] == "chain":
                assert p["chunk"] == count


def batch(exe, n, *ops, **env):
    """Plan ops as one group (plan_test batch mode): one dict per launch."""
    e = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    e.update({k: str(v) for k, v in env.items()})
    out = subprocess.run([exe, str(n), "batch", *ops], env=e, capture_output=True, text=True, timeout=30)
    assert out.returncode == 0, out.stdout + out.stderr
    launches = []
    for line in out.stdout.split("\n"):
        if not line:
            continue
        d = dict(t.split("=") for t in line.split())
        d["ranges"] = [tuple(int(x) for x in r.split("+")) for r in d["ranges"].split(",")]
        if "masks" in d:
            d["masks"] = [int(m, 16) for m in d["masks"].split(",")]
        d["ops"], d["grid"] = int(d["ops"]), int(d["grid"])
        launches.append(d)
    return launches


def test_group_batches_by_kernel_type_and_operator(exe):
    """Group aggregation (enqueue.cc batchable / launchBatch; reference enqueue.cc:405-440): consecutive ops
    planned onto the same kernel with the same type and operator share one launch; the launch's channel ranges
    stay inside its grid and are disjoint while the grid has room for every op."""
    rs = [f"rs:9:{2 * c}" for c in (100, 2000, 8192, 30_000, 100_000, 300_000, 70_000, 1_000_000)]
    got = batch(exe, 2, *rs, "ag:7:5000", "ar:7:1000:2", "ar:7:3:2", "reduce:7:100",
                "ar:7:40000", "ar:7:100000", "ar:7:250000", "ar:7:1000000", "ar:7:600000:2")
    assert [(l["algo"], l["ops"]) for l in got] == [("ll", 4), ("direct", 4), ("ll", 3), ("ll", 1), ("oneshot", 3),
                                                    ("direct", 1), ("direct", 1)]
    for l in got:
        cap = 32 if l["algo"] == "ll" else 256
        assert 1 <= l["grid"] <= cap
        assert all(0 <= off < l["grid"] and 1 <= nch <= l["grid"] for off, nch in l["ranges"]), l
        if sum(nch for _, nch in l["ranges"]) <= l["grid"]:
            used = [c for off, nch in l["ranges"] for c in range(off, off + nch)]
            assert len(used) == len(set(used)), l


def test_ll_batch_channel_masks(exe):
    """An LL batch's per-channel op masks (LLArgs::chMask, launchBatch) say exactly which ops each channel runs: bit k
    of channel c is set iff c is in op k's range (mod the 32 LL channels), wrap-around included, and no channel
    outside the grid has work."""
    for n, ops in ((2, ["ar:7:100", "ar:7:20000", "rs:7:9000", "ag:7:3000", "ar:7:1"] * 4),
                   (8, ["ar:7:100"] * 32), (4, ["ar:9:20000", "ar:9:12", "ar:9:30000"] * 3)):
        ll = [l for l in batch(exe, n, *ops) if l["algo"] == "ll" and l["ops"] > 1]
        assert ll, (n, ops)
        for l in ll:
            want = [0] * 32
            for k, (off, nch) in enumerate(l["ranges"]):
                for j in range(nch):
                    want[(off + j) % 32] |= 1 << k
            assert l["masks"] == want, l
            assert all(m == 0 for m in l["masks"][l["grid"]:]), l


def test_group_batch_limits_and_opt_out(exe):
    # at most 8 staged ops per launch (kMaxCollBatch), 32 LL ops (kMaxLLBatch)
    got = batch(exe, 4, *(["ar:7:100000"] * 10))
    assert [(l["algo"], l["ops"]) for l in got] == [("oneshot", 8), ("oneshot", 2)]
    assert [l["ops"] for l in batch(exe, 8, *(["ar:7:100"] * 40))] == [32, 8]
    # wrap-around once the ops need more channels than the grid: ranges stay in bounds
    big = batch(exe, 2, *(["rs:7:40000000"] * 4))
    assert big[0]["ops"] == 4 and big[0]["grid"] == 256
    assert all(0 <= off < 256 for off, _ in big[0]["ranges"])
    # different types never share a launch; NCCL_AMD_NO_AGGREGATION=1 launches every op alone
    assert [l["ops"] for l in batch(exe, 2, "ar:7:100", "ar:9:100", "ar:7:100")] == [1, 1, 1]
    assert [l["ops"] for l in batch(exe, 2, *(["ar:7:100"] * 3), NCCL_AMD_NO_AGGREGATION=1)] == [1, 1, 1]
    # forced ring / chain plans are not batched (their own kernel)
    assert [l["ops"] for l in batch(exe, 4, *(["ar:7:1000000"] * 3), NCCL_ALGO="RING")] == [1, 1, 1]


def test_ll128_class_protocol(exe):
    # LL128 class (LL64 lines of 56 payload bytes): off by default (the reference too, where 128-byte store
    # atomicity is unproven); NCCL_PROTO=LL128 forces it for everything that fits 32 channels x 512 lines,
    # NCCL_AMD_LL128=1 gives it the size-table range between LL and one-shot (default up to 1 MiB / n)
    assert plan(exe, 2, "ar", 7, (512 << 10) // 4)["algo"] == "oneshot"
    p = plan(exe, 2, "ar", 7, (512 << 10) // 4, NCCL_PROTO="LL128")
    assert p["algo"] == "ll128" and p["part"] * 64 <= 32 << 10 and p["part"] * p["nch"] * 56 >= 512 << 10
    cap_lines = 32 * (32 << 10) // 64
    assert plan(exe, 2, "ar", 9, cap_lines * 56 // 2, NCCL_PROTO="LL128")["algo"] == "ll128"   # exactly full
    assert plan(exe, 2, "ar", 9, cap_lines * 56 // 2 + 28, NCCL_PROTO="LL128")["algo"] != "ll128"
    for n in (2, 4, 8):
        lim = max(64 << 10, (1 << 20) // n)
        assert plan(exe, n, "ar", 7, (16 << 10) // 4, NCCL_AMD_LL128=1)["algo"] == "ll"      # LL range first
        assert plan(exe, n, "ar", 7, lim // 4, NCCL_AMD_LL128=1)["algo"] == "ll128"
        assert plan(exe, n, "ar", 7, lim // 4 + 4, NCCL_AMD_LL128=1)["algo"] in ("oneshot", "direct")
    assert plan(exe, 2, "ar", 7, 100_000, NCCL_AMD_LL128=1, NCCL_PROTO="^LL128")["algo"] == "oneshot"
    assert plan(exe, 2, "ar", 7, 100, NCCL_PROTO="LL,LL128")["algo"] == "ll"    # LL range, Simple off
    assert plan(exe, 2, "ar", 7, 100_000, NCCL_PROTO="LL,LL128")["algo"] == "ll128"
    for func in ("rs", "ag", "reduce"):
        assert plan(exe, 4, func, 7, 20_000, NCCL_PROTO="LL128")["algo"] == "ll128"
    assert plan(exe, 4, "rs", 7, 20_001, NCCL_PROTO="LL128")["algo"] == "direct"  # 8-byte rank blocks only
    # every channel carries at least one line
    for count in (1, 14, 15, 1000, 123_457):
        p = plan(exe, 3, "ar", 7, count, NCCL_PROTO="LL128", NCCL_AMD_LL128_CHANNEL_BYTES=56)
        lines = -(-count * 4 // 56)
        assert (p["nch"] - 1) * p["part"] < lines <= p["nch"] * p["part"]


@pytest.mark.parametrize("n,want", [(2, 256), (3, 64), (4, 64), (5, 128), (7, 128), (8, 128)])
def test_link_channel_budget(exe, n, want):
    """large staged plans at n >= 3 take a CU budget from the link cost model
    (enqueue.cc linkChannelBudget: (2.5n-1) x 76.8 GB/s of HBM traffic / 23 GB/s per staged-kernel workgroup x 2,
    rounded up to a power of two >= 32) instead of every channel; n = 2 keeps all of them."""
    assert plan(exe, n, "ar", 7, (256 << 20) // 4)["nch"] == want
    if n >= 3:
        assert plan(exe, n, "rs", 9, (1 << 30) // 2 // n)["nch"] == want        # C3's ReduceScatter
        assert plan(exe, n, "ag", 9, (1 << 30) // 2 // n)["nch"] == want        # and AllGather
        # NCCL_MAX_CTAS (reference env.rst:901) or NCCL_AMD_LINK_CHANNELS overrule the budget
        assert plan(exe, n, "ar", 7, (256 << 20) // 4, NCCL_MAX_CTAS=256)["nch"] == 256
        assert plan(exe, n, "ar", 7, (256 << 20) // 4, NCCL_AMD_LINK_CHANNELS=0)["nch"] == 256
        assert plan(exe, n, "ar", 7, (256 << 20) // 4, NCCL_AMD_LINK_CHANNELS=16)["nch"] == 16
        # the co-residency cap still applies below the budget (several ranks per GPU)
        assert plan(exe, n, "ar", 7, (256 << 20) // 4, chancap=24)["nch"] == 24


def test_reference_order_direct_allreduce(exe, built):
    """NCCL_AMD_REF_ORDER=1: every AllReduce — the smallest included, no LL / one-shot — runs the direct kernel on the
    reference's ring partition (the same parts and chunk as NCCL_ALGO=RING), other collectives keep their plans."""
    import oracle
    for n, dt, count, k, buff in ((2, 7, 1, 256, None), (2, 7, 1000, 256, None), (3, 6, 100_003, 7, 16384),
                                  (8, 9, 1 << 27, 32, None), (4, 0, 5_000_000, 64, 65536), (8, 7, 1 << 22, 1, None)):
        env = {"NCCL_AMD_REF_ORDER": 1}
        if buff:
            env["NCCL_BUFFSIZE"] = buff
        p = plan(exe, n, "ar", dt, count, chancap=k, **env)
        want = oracle.ring_nccl_plan(count, SIZES[dt], n, min(k, 64), buff or 0)
        assert p["algo"] == "direct", p
        assert (p["refnch"], p["cbdlo"], p["part"], p["cbdhi"], p["chunk"]) == want, (n, dt, count, k, buff, p)
        assert 0 < p["slice"] <= p["chunk"]
    # NCCL_PROTO naming LL or LL128 alone: that protocol's ring partition (its cells, channel shrink and chunk, with
    # NCCL_LL_BUFFSIZE / NCCL_LL128_BUFFSIZE), still on the direct kernel (no LL kernel in this mode)
    import numpy as np
    rng = np.random.default_rng(11)
    counts = [1, 1000, 100_003, 1 << 22] + [int(x) for x in rng.integers(1, 1 << 25, 6)]
    for proto, var, pid, buffs in (("LL", "NCCL_LL_BUFFSIZE", oracle.PROTO_LL, (None, 4096, 65536)),
                                   ("LL128", "NCCL_LL128_BUFFSIZE", oracle.PROTO_LL128, (None, 32768)),
                                   ("^LL,LL128", "NCCL_BUFFSIZE", oracle.PROTO_SIMPLE, (None, 16384))):
        for count in counts:
            for n, dt, k in ((2, 7, 256), (3, 6, 7), (8, 9, 32), (4, 0, 1)):
                for buff in buffs:
                    env = {"NCCL_AMD_REF_ORDER": 1, "NCCL_PROTO": proto}
                    if buff:
                        env[var] = buff
                    p = plan(exe, n, "ar", dt, count, chancap=k, **env)
                    want = oracle.ring_nccl_plan(count, SIZES[dt], n, min(k, 64), buff or 0, pid)
                    assert p["algo"] == "direct", (proto, p)
                    assert (p["refnch"], p["cbdlo"], p["part"], p["cbdhi"], p["chunk"]) == want, (proto, count, n, dt, k, buff, p)
                    assert 0 < p["slice"] <= p["chunk"]
    # NCCL_ALGO=RING with LL or LL128 alone: the ring kernel on that protocol's partition (no LL kernel)
    for proto, pid in (("LL", oracle.PROTO_LL), ("LL128", oracle.PROTO_LL128)):
        for count in (1, 1000, 100_003, 1 << 22):
            p = plan(exe, 3, "ar", 7, count, chancap=7, NCCL_ALGO="RING", NCCL_PROTO=proto)
            assert p["algo"] == "ring", (proto, p)
            assert (p["refnch"], p["cbdlo"], p["part"], p["cbdhi"], p["chunk"]) == \
                oracle.ring_nccl_plan(count, 4, 3, 7, 0, pid), (proto, count, p)
    assert plan(exe, 3, "ar", 7, 1000, NCCL_ALGO="RING", NCCL_PROTO="LL,LL128")["algo"] == "ll"
    assert plan(exe, 8, "rs", 7, 8 << 20, NCCL_AMD_REF_ORDER=1)["cbdlo"] == 0
    assert plan(exe, 2, "ar", 7, 1000, NCCL_AMD_REF_ORDER=1, NCCL_ALGO="TREE")["algo"] == "chain"
    # ref-order AllReduces launch alone (never batched)
    assert [l["ops"] for l in batch(exe, 2, *(["ar:7:1000000"] * 3), NCCL_AMD_REF_ORDER=1)] == [1, 1, 1]


def test_ring_allreduce_takes_the_reference_partition(exe, built):
    """NCCL_ALGO=RING AllReduce is planned on the reference's own channel parts and chunk (enqueue.cc ringParts;
    reference enqueue.cc:576-757, 2091-2097, 2222-2321), identical to the C oracle's restatement over a sweep
    of sizes, types, rank counts, channel caps and NCCL_BUFFSIZE values."""
    import numpy as np
    import oracle
    rng = np.random.default_rng(3)
    counts = [1, 7, 4099, 100_003, 1 << 20, 67_108_864] + [int(x) for x in rng.integers(1, 1 << 26, 12)]
    for count in counts:
        for dt in (0, 6, 7, 8):
            for n, k in ((2, 256), (3, 7), (8, 32), (4, 1)):
                for buff in (None, 16384):
                    env = {"NCCL_ALGO": "RING"}
                    if buff:
                        env["NCCL_BUFFSIZE"] = buff
                    p = plan(exe, n, "ar", dt, count, chancap=k, **env)
                    want = oracle.ring_nccl_plan(count, SIZES[dt], n, min(k, 64), buff or 0)
                    assert p["algo"] == "ring", p
                    assert (p["refnch"], p["cbdlo"], p["part"], p["cbdhi"], p["chunk"]) == want, (count, dt, n, k, buff)
                    assert 0 < p["slice"] <= p["chunk"] and p["slice"] % (16 // SIZES[dt]) == 0


def test_reference_partition_is_clamped_and_decoupled(exe, built):
    """the reference never runs more than MAXCHANNELS = 64 channels (src/include/device.h:91),
    so NCCL_AMD_REF_ORDER / NCCL_ALGO=RING walk at most 64 reference parts (NCCL_AMD_REF_NCHANNELS names the
    reference run's K; the channel cap otherwise), and refSub workgroups share each part, so the launch fills the
    channel cap whatever K is: K = 32 at 256 MiB fp32, n = 2 runs 32 parts x 8 workgroups = 256."""
    import oracle
    S = (256 << 20) // 4
    for env in ({"NCCL_AMD_REF_ORDER": 1}, {"NCCL_ALGO": "RING"}):
        p = plan(exe, 2, "ar", 7, S, **env)                                     # cap 256 -> K = 64
        assert (p["refnch"], p["cbdlo"], p["part"], p["cbdhi"], p["chunk"]) == oracle.ring_nccl_plan(S, 4, 2, 64, 0)
        assert p["sub"] == 4 and p["nch"] == 256
        p = plan(exe, 2, "ar", 7, S, NCCL_AMD_REF_NCHANNELS=32, **env)          # the reference run's K = 32
        assert (p["refnch"], p["cbdlo"], p["part"], p["cbdhi"], p["chunk"]) == oracle.ring_nccl_plan(S, 4, 2, 32, 0)
        assert p["sub"] == 8 and p["nch"] == 256
        p = plan(exe, 2, "ar", 7, S, NCCL_AMD_REF_NCHANNELS=200, **env)         # clamped
        assert p["refnch"] == 64
        p = plan(exe, 2, "ar", 7, S, chancap=32, **env)                          # NCCL_MAX_CTAS=32: 32 workgroups
        assert p["refnch"] == 32 and p["sub"] == 1 and p["nch"] == 32
        p = plan(exe, 3, "ar", 7, S, chancap=3, NCCL_AMD_REF_NCHANNELS=5, **env)  # a part per workgroup at least:
        assert p["refnch"] == 3 and p["nch"] == 3                                 # K clamped to the channel cap
        assert (p["refnch"], p["cbdlo"], p["part"], p["cbdhi"], p["chunk"]) == oracle.ring_nccl_plan(S, 4, 3, 3, 0)
    # small messages: no sub-chunk below the default plan's 16 KiB granularity, never more than the channel cap
    for count in (1, 1000, 100_003, 1 << 20, 3_000_001):
        for n in (2, 3, 8):
            p = plan(exe, n, "ar", 7, count, NCCL_AMD_REF_ORDER=1, NCCL_AMD_REF_NCHANNELS=16)
            assert p["nch"] == p["refnch"] * p["sub"] and 1 <= p["nch"] <= 256
            ck = min(p["chunk"], -(-(max(p["cbdlo"], p["part"], p["cbdhi"]) // 1) // n))
            assert p["sub"] == 1 or -(-ck // p["sub"]) * 4 >= (16 << 10) - 16, (count, n, p)
            if n >= 3:  # the CU budget of the default plan at n >= 3 (linkChannelBudget: 64 at n = 3, 128 at n = 8)
                assert p["nch"] <= max({3: 64, 8: 128}[n], p["refnch"])


def test_size_table_file(exe, tmp_path):
    """the LL / LL128-class / one-shot crossovers come from a per-n table that
    NCCL_AMD_SIZE_TABLE=<file> overrides (reference: the tuning tables behind the cost model, src/graph/tuning.cc:
    148-212, 630-655), so a measured 8-GPU sweep is adopted without a rebuild. The built-in rows are pinned by
    test_allreduce_size_table; here the file's syntax, precedence and error handling."""
    t = tmp_path / "table.txt"
    t.write_text("# nranks ll ll128 oneshot\n"
                 "*   -    -     1M      # every n: one-shot to 1 MiB\n"
                 "8   48K  -     512K    # n = 8 row overrides the '*' row\n"
                 "2   64k  2M    -\n")
    tab = dict(NCCL_AMD_SIZE_TABLE=str(t))
    # n = 8: LL to 48 KiB (built-in 32 KiB), one-shot to 512 KiB (built-in 256 KiB)
    assert plan(exe, 8, "ar", 7, (48 << 10) // 4, **tab)["algo"] == "ll"
    assert plan(exe, 8, "ar", 7, (48 << 10) // 4 + 4, **tab)["algo"] == "oneshot"
    assert plan(exe, 8, "ar", 7, (512 << 10) // 4, **tab)["algo"] == "oneshot"
    assert plan(exe, 8, "ar", 7, (512 << 10) // 4 + 4, **tab)["algo"] == "direct"
    assert plan(exe, 8, "ar", 7, (512 << 10) // 4)["algo"] == "direct"          # built-in: 256 KiB
    # n = 4 takes the '*' row: one-shot to 1 MiB (built-in 512 KiB), LL unchanged (64 KiB)
    assert plan(exe, 4, "ar", 7, (1 << 20) // 4, **tab)["algo"] == "oneshot"
    assert plan(exe, 4, "ar", 7, (64 << 10) // 4, **tab)["algo"] == "ll"
    assert plan(exe, 4, "ar", 7, (64 << 10) // 4 + 4, **tab)["algo"] == "oneshot"
    # n = 2: LL to 64 KiB (built-in 128 KiB); its '-' one-shot keeps the '*' row's 1 MiB
    assert plan(exe, 2, "ar", 7, (64 << 10) // 4 + 4, **tab)["algo"] == "oneshot"
    assert plan(exe, 2, "ar", 7, (2 << 20) // 4, **tab)["algo"] == "direct"
    # the LL128 class range (when enabled) from the table: n = 2 up to 2 MiB, within the line area (~896 KiB)
    assert plan(exe, 2, "ar", 7, (768 << 10) // 4, NCCL_AMD_LL128=1, **tab)["algo"] == "ll128"
    assert plan(exe, 2, "ar", 7, (768 << 10) // 4, NCCL_AMD_LL128=1)["algo"] == "oneshot"   # built-in: 512 KiB
    # the explicit knobs still win over the table
    assert plan(exe, 8, "ar", 7, (512 << 10) // 4, NCCL_AMD_ONESHOT_BYTES=1 << 20, **tab)["algo"] == "oneshot"
    assert plan(exe, 8, "ar", 7, (40 << 10) // 4, NCCL_AMD_LL_BYTES=1024, **tab)["algo"] == "oneshot"


def test_size_table_bad_lines_are_ignored(exe, tmp_path):
    t = tmp_path / "bad.txt"
    t.write_text("8 48K\n"              # too few columns
                 "x 1K 1K 1K\n"         # not a rank count
                 "99 1K 1K 1K\n"        # out of range
                 "8 1Q 1K 1K\n"         # bad size
                 "8 nan 1K 1K\n"        # not finite (strtod accepts it)
                 "8 1K inf -\n"
                 "8 - - 512K\n")        # the one good row
    e = dict(NCCL_AMD_SIZE_TABLE=str(t), NCCL_DEBUG="WARN")
    assert plan(exe, 8, "ar", 7, (512 << 10) // 4, **e)["algo"] == "oneshot"
    assert plan(exe, 8, "ar", 7, (32 << 10) // 4, **e)["algo"] == "ll"          # built-in LL row kept
    out = subprocess.run([exe, "8", "ar", "7", "1000"], env=dict(os.environ, **e), capture_output=True, text=True)
    assert out.stderr.count("line ignored") + out.stdout.count("line ignored") == 6, out.stdout + out.stderr
    # an unreadable file: the built-in table, with a warning
    assert plan(exe, 8, "ar", 7, (256 << 10) // 4, NCCL_AMD_SIZE_TABLE=str(tmp_path / "none"))["algo"] == "oneshot"


def test_size_table_zero_and_huge_sizes(exe, tmp_path):
    # 0 is a size (no LL at n = 8: one-shot from the first byte), '-' keeps the built-in value; a size beyond any buffer
    # saturates instead of overflowing (one-shot at every size for n = 4)
    t = tmp_path / "edge.txt"
    t.write_text("8 0 - -\n4 - - 1e30\n")
    tab = dict(NCCL_AMD_SIZE_TABLE=str(t))
    assert plan(exe, 8, "ar", 7, 8, **tab)["algo"] == "oneshot"
    assert plan(exe, 8, "ar", 7, 8)["algo"] == "ll"
    assert plan(exe, 8, "ar", 7, (1 << 20) // 4, **tab)["algo"] == "direct"          # its one-shot row kept
    assert plan(exe, 4, "ar", 7, (64 << 20) // 4, **tab)["algo"] == "oneshot"
    assert plan(exe, 4, "ar", 7, 8, **tab)["algo"] == "ll"


@pytest.mark.parametrize("n", [2, 3, 4, 5, 6, 7, 8, 16])
def test_channel_peer_order_is_a_latin_square(exe, n):
    """every workgroup-wide multi-peer loop (staged scatter, pull gather, zero-copy pulls) visits
    the peers in device_abi.h chanPeer's channel-rotated order. For every rank and step position k, any n-1
    consecutive channels visit all n-1 peers once, so over K channels each peer carries floor or ceil(K/(n-1)) of
    them (at K = 128, n = 8: 18-19 channels on each of the 7 links at every step position, instead of 128 on one);
    and for a fixed (channel, k) the ranks' choices are a permutation: no rank's link is read by two ranks."""
    for K in (1, n - 1, 64, 128, 256):
        out = subprocess.run([exe, "peers", str(n), str(K)], capture_output=True, text=True, timeout=30)
        assert out.returncode == 0, out.stderr
        order = {}
        for line in out.stdout.split("\n"):
            if line:
                me, c, *ps = map(int, line.split())
                order[me, c] = ps
        assert len(order) == n * K
        for me in range(n):
            peers = set(range(n)) - {me}
            for c in range(K):
                assert sorted(order[me, c]) == sorted(peers), (me, c)        # every peer once per channel
            for k in range(n - 1):
                col = [order[me, c][k] for c in range(K)]
                for c0 in range(0, K - (n - 1) + 1):
                    assert set(col[c0:c0 + n - 1]) == peers, (me, k, c0)    # Latin: any n-1 channels cover all
                counts = [col.count(p) for p in peers]
                assert max(counts) - min(counts) <= 1 and sum(counts) == K, (me, k, counts)
        for c in range(K):
            for k in range(n - 1):
                assert sorted(order[me, c][k] for me in range(n)) == list(range(n)), (c, k)


def test_eager_registration_eligibility(exe):
    """with NCCL_AMD_EAGER_REGISTER=1 an unregistered collective of at least
    NCCL_AMD_EAGER_REGISTER_BYTES whose staged plan would be the direct kernel registers its allocations on first use
    and runs the zero-copy kernel (the stub's registration always succeeds). The decision uses only what every rank
    shares (bytes, the size table), so every rank takes the same kernel."""
    on = dict(NCCL_AMD_EAGER_REGISTER=1)
    S = (256 << 20) // 4
    assert plan(exe, 2, "ar", 7, S)["algo"] == "direct"                       # default: off
    assert plan(exe, 2, "ar", 7, S, PLAN_MULTIPROCESS=1)["algo"] == "direct"  # ... across processes too
    # -1: on for communicators spanning processes (every peer serving registrations), off within one process
    auto = dict(NCCL_AMD_EAGER_REGISTER=-1)
    assert plan(exe, 2, "ar", 7, S, PLAN_MULTIPROCESS=1, **auto)["algo"] == "sym"
    assert plan(exe, 8, "rs", 7, S // 8, PLAN_MULTIPROCESS=1, **auto)["algo"] == "sym"
    assert plan(exe, 2, "ar", 7, S, **auto)["algo"] == "direct"
    assert plan(exe, 2, "ar", 7, (1 << 20) // 4, PLAN_MULTIPROCESS=1, **auto)["algo"] == "oneshot"
    assert plan(exe, 2, "ar", 7, S, **on)["algo"] == "sym"
    assert plan(exe, 8, "ar", 7, S, **on)["algo"] == "sym"
    assert plan(exe, 8, "rs", 7, S // 8, **on)["algo"] == "sym"
    assert plan(exe, 8, "ag", 7, S // 8, **on)["algo"] == "sym"
    assert plan(exe, 8, "reduce", 7, S, **on)["algo"] == "direct"            # Reduce keeps the staged path
    assert plan(exe, 2, "ar", 7, (1 << 20) // 4, **on)["algo"] == "oneshot"  # one-shot range: staged
    assert plan(exe, 8, "ar", 7, (1 << 20) // 4, **on)["algo"] == "sym"      # above n = 8's one-shot range
    assert plan(exe, 8, "ar", 7, (512 << 10) // 4, **on)["algo"] == "direct" # below the 1 MiB default threshold
    assert plan(exe, 8, "ar", 7, (512 << 10) // 4, NCCL_AMD_EAGER_REGISTER_BYTES=256 << 10, **on)["algo"] == "sym"
    assert plan(exe, 2, "ar", 7, 1000, **on)["algo"] == "ll"                 # LL range: untouched
    assert plan(exe, 1, "ar", 7, S, **on)["algo"] == "copy"                  # one rank: nothing to register
    assert plan(exe, 2, "ar", 7, S, NCCL_ALGO="RING", **on)["algo"] == "ring"  # forced reference algorithms win
