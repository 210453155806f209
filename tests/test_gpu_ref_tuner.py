"""The tuner boundary pinned by the reference's OWN tuner plugins, unmodified: oracle/Makefile
compiles /root/reference/plugins/tuner/example/plugin.c (exports ncclTunerPlugin_v6 / _v5, reads
NCCL_TUNER_CONFIG_FILE: plugins/tuner/example/plugin.c:335, 504-520) and plugins/tuner/basic/plugin.c (exports
ncclTunerPlugin_v4 only: basic/plugin.c:30) with their own nccl/ headers into oracle/_ref/. Loaded into libnccl.so
through NCCL_TUNER_PLUGIN (reference src/plugin/tuner.cc: v6 -> v5 -> v4), each must steer the algorithm, protocol
and channel count as its config says — seen in the kernel log (NCCL_AMD_KERNEL_LOG: every distinct kernel and grid
launched) — while every result stays bit-exact against the oracle.

The example plugin's CSV (the reference's format, plugins/tuner/example/nccl_tuner.conf) is written by the test: one
size band per algorithm / protocol / channel choice this engine maps ((RING|TREE, LL) -> LL,
(TREE, SIMPLE) -> one-shot, (RING, SIMPLE) -> direct)."""
import multiprocessing as mp
import os
import queue

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")

CONF = """# collective_type,min_bytes,max_bytes,algorithm,protocol,channels,nNodes,nRanks
allreduce,0,8192,ring,ll,2,1,2
allreduce,8193,524288,tree,simple,4,1,2
allreduce,524289,4294967295,ring,simple,6,1,2
reducescatter,0,4294967295,ring,simple,3,-1,-1
allgather,0,65536,ring,ll,5,-1,-1
reduce,0,4294967295,ring,simple,7,-1,-1
"""
# (collective, count as gpu_cases.run_case takes it, root)
CASES = [("allreduce", 1024, 0), ("allreduce", 65_536, 0), ("allreduce", 1 << 20, 0),
         ("reducescatter", 2 * 50_000, 0), ("allgather", 4096, 0), ("reduce", 300_001, 1)]
# what the example plugin's config must launch for each case (kernel name fragment, grid)
WANT_EXAMPLE = [("::llKernel", 2), ("collKernel<float, 0, 4>", 4), ("collKernel<float, 0, 0>", 6),
                ("collKernel<float, 0, 1>", 3), ("::llKernel", 5), ("collKernel<float, 0, 3>", 7)]


def _worker(plugin, conf, q):
    try:
        os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "30000"
        os.environ["NCCL_TUNER_PLUGIN"] = plugin
        if conf:
            os.environ["NCCL_TUNER_CONFIG_FILE"] = conf
        klog = f"/tmp/nccl_amd_reftuner_kernels_{os.getpid()}.log"
        dlog = f"/tmp/nccl_amd_reftuner_debug_{os.getpid()}.log"
        for f in (klog, dlog):
            if os.path.exists(f):
                os.remove(f)
        os.environ["NCCL_AMD_KERNEL_LOG"] = klog
        os.environ["NCCL_DEBUG"] = "INFO"
        os.environ["NCCL_DEBUG_FILE"] = dlog
        import torch
        import nccl_amd
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0])
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        cs = list(zip(comms, streams))
        errs, launched = [], []
        for i, (coll, count, root) in enumerate(CASES):
            if os.path.exists(klog):
                os.remove(klog)
            # the kernel log names each distinct (kernel, grid) once per process: the case's own launch
            errs += G.run_case(cs, coll, 7, 0, count, 0, seed=740 + i, root=root)
            torch.cuda.synchronize()
            launched.append(open(klog).read().splitlines() if os.path.exists(klog) else [])
        for c in comms:
            c.destroy()
        q.put((errs, launched, open(dlog).read() if os.path.exists(dlog) else ""))
    except Exception as e:
        q.put(([f"exception {e!r}"], [], ""))


def _run(plugin, conf=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(plugin, conf, q))
    p.start()
    try:
        out = q.get(timeout=240)
    except queue.Empty:
        p.kill()
        raise AssertionError("tuner worker timed out")
    p.join(timeout=60)
    return out


def _need(path):
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: build it with `make -C oracle ref` (needs /root/reference) before the GPU run")


def _first(lines, frag):
    return [ln for ln in lines if frag in ln]


def test_reference_example_tuner_v6(built, tmp_path):
    """The reference's example plugin (v6) with a config forcing LL / one-shot / direct and a channel count per size
    band: each choice takes effect, bit-exact."""
    plugin = os.path.join(REF, "libnccl-tuner-example.so")
    _need(plugin)
    conf = tmp_path / "nccl_tuner.conf"
    conf.write_text(CONF)
    errs, launched, log = _run(plugin, str(conf))
    assert not errs, "\n".join(errs[:20])
    assert "TUNER/Plugin: loaded" in log and "TUNER/ExamplePlugin: Loaded 6 tuning configurations" in log, log[-3000:]
    for (coll, count, _), (frag, grid), lines in zip(CASES, WANT_EXAMPLE, launched):
        hit = [ln for ln in _first(lines, frag) if f" grid={grid} " in ln]
        assert hit, f"{coll} count {count}: want {frag} grid={grid}, launched {lines}"
    assert log.count("TUNER/ExamplePlugin: Applied config") >= len(CASES), log[-3000:]


def test_reference_example_tuner_without_config(built, tmp_path):
    """No config file: the example plugin leaves the cost table alone and returns nChannels = 1 (its default,
    plugin.c:360), so the engine's size table picks the kernel and the reference's nMaxChannels = 1 limits it to one
    workgroup (enqueue.cc:2189) — still bit-exact."""
    plugin = os.path.join(REF, "libnccl-tuner-example.so")
    _need(plugin)
    errs, launched, log = _run(plugin, str(tmp_path / "absent.conf"))
    assert not errs, "\n".join(errs[:20])
    big = launched[2]  # 4 MiB AllReduce: the size table's direct kernel, on one channel
    assert _first(big, "collKernel<float, 0, 0>") and all(" grid=1 " in ln for ln in big), big


def test_reference_basic_tuner_v4(built):
    """The reference's basic plugin exports only ncclTunerPlugin_v4, so it loads through the fallback; it makes
    (RING, SIMPLE) free and asks for one channel, so every collective — the LL-sized ones included — runs the direct
    kernel on one workgroup, bit-exact."""
    plugin = os.path.join(REF, "libnccl-tuner-basic.so")
    _need(plugin)
    errs, launched, log = _run(plugin)
    assert not errs, "\n".join(errs[:20])
    assert "TUNER/Plugin: loaded" in log, log[-3000:]
    seen = [ln for lines in launched for ln in lines]  # each distinct (kernel, grid) is logged once per process
    assert not any("::llKernel" in ln for ln in seen), seen
    assert seen and all(" grid=1 " in ln for ln in seen), seen
    for frag in ("collKernel<float, 0, 0>", "collKernel<float, 0, 1>", "collKernel<unsigned int, 0, 2>",
                 "collKernel<float, 0, 3>"):
        assert _first(seen, frag), f"want {frag} on one workgroup, launched {seen}"


CONF_REGBUFF = """# the reference CSV's optional 9th / 10th columns: numPipeOps, regBuff
allreduce,0,4294967295,ring,simple,6,-1,-1,-1,0
allreduce,0,4294967295,tree,simple,4,-1,-1,-1,1
"""


def _regbuff_worker(plugin, conf, q):
    try:
        os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
        os.environ["NCCL_AMD_SPIN_TIMEOUT_MS"] = "30000"
        os.environ["NCCL_TUNER_PLUGIN"] = plugin
        os.environ["NCCL_TUNER_CONFIG_FILE"] = conf
        klog = f"/tmp/nccl_amd_reftuner_reg_{os.getpid()}.log"
        if os.path.exists(klog):
            os.remove(klog)
        os.environ["NCCL_AMD_KERNEL_LOG"] = klog
        import torch
        import nccl_amd
        import oracle
        from tests import gpu_cases as G
        torch.cuda.set_device(0)
        comms = nccl_amd.Communicator.init_all([0, 0])
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        count = 3 << 20
        errs, launched = [], []
        for registered in (False, True):
            ins = G.make_inputs(2, 7, count, seed=760 + registered)
            xs = [torch.from_numpy(a).cuda() for a in ins]
            ys = [torch.empty_like(x) for x in xs]
            hs = ([c.register_buffer(b.data_ptr(), count * 4) for c, x, y in zip(comms, xs, ys) for b in (x, y)]
                  if registered else [])
            torch.cuda.synchronize()
            if os.path.exists(klog):
                os.remove(klog)
            with nccl_amd.group():
                for c, s, x, y in zip(comms, streams, xs, ys):
                    c.all_reduce_raw(x.data_ptr(), y.data_ptr(), count, 7, 0, s.cuda_stream)
            torch.cuda.synchronize()
            launched.append(open(klog).read().splitlines() if os.path.exists(klog) else [])
            want = oracle.all_reduce(ins, 7, 0)
            for r, y in enumerate(ys):
                if not G.same_bits(y.cpu().numpy(), want, 7):
                    errs.append(f"registered={registered} rank {r}: differs")
            for i, h in enumerate(hs):
                comms[i // 2].deregister_buffer(h)
        for c in comms:
            c.destroy()
        q.put((errs, launched, ""))
    except Exception as e:
        q.put(([f"exception {e!r}"], [], ""))


def test_reference_example_tuner_sees_regbuff(built, tmp_path):
    """The plugin gets the reference's regBuff (enqueue.cc:2141-2147: both buffers registered): the example plugin's
    regBuff column picks RING/SIMPLE on 6 channels for unregistered buffers (the staged direct kernel) and TREE/SIMPLE
    on 4 for registered ones (the zero-copy kernel, on the plugin's 4 channels), bit-exact."""
    plugin = os.path.join(REF, "libnccl-tuner-example.so")
    _need(plugin)
    conf = tmp_path / "regbuff.conf"
    conf.write_text(CONF_REGBUFF)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_regbuff_worker, args=(plugin, str(conf), q))
    p.start()
    try:
        errs, launched, _ = q.get(timeout=240)
    except queue.Empty:
        p.kill()
        raise AssertionError("tuner worker timed out")
    p.join(timeout=60)
    assert not errs, "\n".join(errs)
    assert any("collKernel<float, 0, 0>" in ln and " grid=6 " in ln for ln in launched[0]), launched
    assert any("symKernel" in ln and " grid=4 " in ln for ln in launched[1]), launched
