"""GPU checks of the kernels' 1-byte element arithmetic, exhaustively:

* tests/native/fp8_cvt_probe: the hardware fp8 conversions the kernels use (numerics.h fp8ToF32Hw /
  f32ToFp8SatHw: v_cvt_f32_fp8 / v_cvt_pk_fp8_f32 with a satfinite clamp and software NaN) equal the software
  conversions (checked against the oracle on the host, tests/test_numerics.py) for every code and every half;
* every (a, b) byte pair of e4m3 / e5m2 / uint8 / int8 through an n=2 AllReduce (both ranks on the one GPU)
  for every operator, on the LL kernel and on the staged kernel, bit-exact vs the oracle — the reference's
  fp8 functors (src/device/reduce_kernel.h:461-487) and integer functors (:330-357, :936-966)."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fp8_convert_probe(built):
    exe = os.path.join(ROOT, "tests", "native", "fp8_cvt_probe")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    for fmt in ("e4m3", "e5m2"):
        assert r[f"{fmt}_decode_mismatch"] == 0 and r[f"{fmt}_encode_mismatch"] == 0, r


def test_fp8_packed_half_probe(built):
    """The packed fp8 <-> half converts the packed-half fold runs on (numerics.h fp8DecodeH2 / fp8RoundH2): decode
    exact for every code, clamped encode exact for every non-NaN half (NaN packs take the f32 path)."""
    exe = os.path.join(ROOT, "tests", "native", "fp8_f16_probe")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    for fmt in ("e4m3", "e5m2"):
        assert r[f"{fmt}_decode_mismatch"] == 0 and r[f"{fmt}_encode_clamped_mismatch"] == 0, r


def _pairs(dtype):
    a = np.repeat(np.arange(256, dtype=np.uint8), 256)
    b = np.tile(np.arange(256, dtype=np.uint8), 256)
    npdt = np.int8 if dtype == 0 else np.uint8
    return [a.view(npdt), b.view(npdt)]


@pytest.mark.parametrize("proto", ["LL", "^LL"])
def test_one_byte_every_pair(built, proto, monkeypatch):
    import torch
    import nccl_amd
    from tests import gpu_cases as G
    monkeypatch.setenv("NCCL_PROTO", proto)
    os.environ["NCCL_MULTI_RANK_GPU_ENABLE"] = "1"
    torch.cuda.set_device(0)
    comms = nccl_amd.Communicator.init_all([0, 0])
    cs = list(zip(comms, [torch.cuda.Stream(), torch.cuda.Stream()]))
    errs = []
    try:
        for dtype in (10, 11, 1, 0):
            ins = _pairs(dtype)
            for op in (0, 1, 2, 3, 4):  # sum, prod, max, min, avg
                errs += G.run_case(cs, "allreduce", dtype, op, ins[0].size, 0, seed=0, inputs=ins)
    finally:
        for c in comms:
            c.destroy()
    assert not errs, "\n".join(errs[:10])
