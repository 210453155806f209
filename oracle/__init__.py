"""oracle — CPU parity checker for the MI355X reduction engine. TEST INFRASTRUCTURE ONLY.

Loads oracle/_build/liboracle.so (built from oracle/nccl_oracle.c by `make oracle`), the C
restatement of the reference's reduction semantics (see the header of nccl_oracle.c for the
reference file:line of every rule). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package; the product (nccl_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

# ncclDataType_t -> numpy storage dtype (small floats are raw bit patterns)
NP_STORAGE = {0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64, 5: np.uint64, 6: np.uint16,
              7: np.float32, 8: np.float64, 9: np.uint16, 10: np.uint8, 11: np.uint8}
DEV_SUM, DEV_PROD, DEV_MINMAX, DEV_PREMULSUM, DEV_SUMPOSTDIV = range(5)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"oracle library {LIB} missing: run `make oracle`")
        L = ctypes.CDLL(LIB)
        P, I, S, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64
        PP = ctypes.POINTER(ctypes.c_void_p)
        L.oracle_host_to_dev_op.argtypes = [I, I, I, ctypes.POINTER(I), ctypes.POINTER(U64)]
        L.oracle_all_reduce.argtypes = [I, I, U64, I, PP, S, P]
        L.oracle_all_reduce_chain.argtypes = [I, I, U64, I, PP, S, P]
        L.oracle_all_reduce_ring_nccl.argtypes = [I, I, U64, I, PP, S, P, I, S]
        L.oracle_ring_nccl_plan.argtypes = [S, I, I, I, S, ctypes.POINTER(U64)]
        L.oracle_all_reduce_ring_nccl_proto.argtypes = [I, I, U64, I, PP, S, P, I, I, S]
        L.oracle_ring_nccl_plan_proto.argtypes = [S, I, I, I, I, S, ctypes.POINTER(U64)]
        L.oracle_reduce_scatter.argtypes = [I, I, U64, I, PP, S, PP]
        L.oracle_reduce.argtypes = [I, I, U64, I, I, PP, S, P]
        L.oracle_fill.argtypes = [I, U64, S, P, I]
        L.oracle_fill_at.argtypes = [I, U64, S, S, P, I]
        L.oracle_cpu_allreduce_f32.argtypes = [I, PP, S, P, I]
        L.oracle_f32_to_f16.argtypes = [ctypes.c_float]
        L.oracle_f32_to_f16.restype = ctypes.c_uint16
        L.oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
        L.oracle_f16_to_f32.restype = ctypes.c_float
        L.oracle_f32_to_bf16.argtypes = [ctypes.c_float]
        L.oracle_f32_to_bf16.restype = ctypes.c_uint16
        L.oracle_bf16_to_f32.argtypes = [ctypes.c_uint16]
        L.oracle_bf16_to_f32.restype = ctypes.c_float
        L.oracle_fp8_to_f32.argtypes = [ctypes.c_uint8, I]
        L.oracle_fp8_to_f32.restype = ctypes.c_float
        L.oracle_f32_to_fp8.argtypes = [ctypes.c_float, I]
        L.oracle_f32_to_fp8.restype = ctypes.c_uint8
        _lib = L
    return _lib


def _ptrs(arrs: Sequence[np.ndarray]):
    a = (ctypes.c_void_p * len(arrs))()
    for i, x in enumerate(arrs):
        a[i] = x.ctypes.data
    return a


def dev_op(op: int, dtype: int, nranks: int):
    d = ctypes.c_int()
    arg = ctypes.c_uint64()
    rc = lib().oracle_host_to_dev_op(op, dtype, nranks, ctypes.byref(d), ctypes.byref(arg))
    if rc:
        raise ValueError(f"invalid op {op} for dtype {dtype}")
    return d.value, arg.value


def all_reduce(inputs: Sequence[np.ndarray], dtype: int, op: int = 0, premul_scalar_bits: int | None = None):
    """Result of ncclAllReduce over `inputs` (one array per rank, storage dtype NP_STORAGE[dtype])."""
    n = len(inputs)
    if premul_scalar_bits is not None:
        d, arg = DEV_PREMULSUM, premul_scalar_bits
    else:
        d, arg = dev_op(op, dtype, n)
    ins = [np.ascontiguousarray(x) for x in inputs]
    out = np.empty_like(ins[0])
    rc = lib().oracle_all_reduce(dtype, d, arg, n, _ptrs(ins), ins[0].size, out.ctypes.data)
    assert rc == 0
    return out


def all_reduce_chain(inputs: Sequence[np.ndarray], dtype: int, op: int = 0):
    """ncclAllReduce with NCCL_ALGO=TREE on one node: the chain 0 <- 1 <- ... <- n-1 (fold order n-1 .. 0)."""
    n = len(inputs)
    d, arg = dev_op(op, dtype, n)
    ins = [np.ascontiguousarray(x) for x in inputs]
    out = np.empty_like(ins[0])
    rc = lib().oracle_all_reduce_chain(dtype, d, arg, n, _ptrs(ins), ins[0].size, out.ctypes.data)
    assert rc == 0
    return out


PROTO_LL, PROTO_LL128, PROTO_SIMPLE = 0, 1, 2  # NCCL_PROTO_* ids (reference device.h)


def ring_nccl_plan(count: int, type_size: int, nranks: int, nchannels: int, buffsize: int = 0,
                   proto: int = PROTO_SIMPLE):
    """The reference's RING AllReduce partition of `count` elements on a communicator of `nchannels` channels
    under protocol `proto` with that protocol's buffer size (0 = its default; nccl_oracle.c
    oracle_ring_nccl_plan_proto): (channels, countLo, countMid, countHi, chunk elements)."""
    plan = (ctypes.c_uint64 * 5)()
    rc = lib().oracle_ring_nccl_plan_proto(count, type_size, nranks, nchannels, proto, buffsize, plan)
    if rc:
        raise ValueError("invalid ring plan arguments")
    return tuple(int(x) for x in plan)


def all_reduce_ring_nccl(inputs: Sequence[np.ndarray], dtype: int, op: int, nchannels: int, buffsize: int = 0,
                         proto: int = PROTO_SIMPLE):
    """ncclAllReduce with NCCL_ALGO=RING in the reference's full-size order for protocol `proto` (Simple by
    default): channel parts, loops of n chunks, last loop re-cut (all_reduce.h:21-81) on a communicator of
    `nchannels` channels."""
    n = len(inputs)
    d, arg = dev_op(op, dtype, n)
    ins = [np.ascontiguousarray(x) for x in inputs]
    out = np.empty_like(ins[0])
    rc = lib().oracle_all_reduce_ring_nccl_proto(dtype, d, arg, n, _ptrs(ins), ins[0].size, out.ctypes.data,
                                                 nchannels, proto, buffsize)
    assert rc == 0
    return out


def reduce_scatter(inputs: Sequence[np.ndarray], dtype: int, op: int = 0, premul_scalar_bits: int | None = None):
    n = len(inputs)
    if premul_scalar_bits is not None:
        d, arg = DEV_PREMULSUM, premul_scalar_bits
    else:
        d, arg = dev_op(op, dtype, n)
    ins = [np.ascontiguousarray(x) for x in inputs]
    rc_count = ins[0].size // n
    outs = [np.empty(rc_count, dtype=ins[0].dtype) for _ in range(n)]
    rc = lib().oracle_reduce_scatter(dtype, d, arg, n, _ptrs(ins), rc_count, _ptrs(outs))
    assert rc == 0
    return outs


def reduce(inputs: Sequence[np.ndarray], dtype: int, op: int, root: int):
    n = len(inputs)
    d, arg = dev_op(op, dtype, n)
    ins = [np.ascontiguousarray(x) for x in inputs]
    out = np.empty_like(ins[0])
    rc = lib().oracle_reduce(dtype, d, arg, n, root, _ptrs(ins), ins[0].size, out.ctypes.data)
    assert rc == 0
    return out


def all_gather(inputs: Sequence[np.ndarray]):
    return np.concatenate([np.ascontiguousarray(x) for x in inputs])


def fill(dtype: int, seed: int, count: int, kind: int = 0) -> np.ndarray:
    """splitmix64 synthetic input: kind 0 uniform [-1,1) / full-range ints, 1 dyadic."""
    out = np.empty(count, dtype=NP_STORAGE[dtype])
    lib().oracle_fill(dtype, seed, count, out.ctypes.data, kind)
    return out


def fill_at(dtype: int, seed: int, start: int, count: int, kind: int = 0) -> np.ndarray:
    """Elements [start, start + count) of fill(dtype, seed, ...) (a rank's slice without the whole buffer)."""
    out = np.empty(count, dtype=NP_STORAGE[dtype])
    lib().oracle_fill_at(dtype, seed, start, count, out.ctypes.data, kind)
    return out


def cpu_allreduce_f32(inputs: Sequence[np.ndarray], nthreads: int = 0):
    """Naive OpenMP CPU baseline; returns (output, threads used)."""
    ins = [np.ascontiguousarray(x, dtype=np.float32) for x in inputs]
    out = np.empty_like(ins[0])
    used = lib().oracle_cpu_allreduce_f32(len(ins), _ptrs(ins), ins[0].size, out.ctypes.data, nthreads)
    return out, used


def to_f32(dtype: int, raw: np.ndarray) -> np.ndarray:
    """Decode storage bits of a small-float type to float32 (oracle conversions)."""
    L = lib()
    if dtype == 7:
        return raw.astype(np.float32)
    if dtype == 8:
        return raw.astype(np.float64)
    if dtype == 6:
        return raw.view(np.float16).astype(np.float32)
    if dtype == 9:
        return (raw.astype(np.uint32) << 16).view(np.float32)
    if dtype in (10, 11):
        table = np.array([L.oracle_fp8_to_f32(i, int(dtype == 11)) for i in range(256)], dtype=np.float32)
        return table[raw]
    return raw.astype(np.float64)


def float_tolerance(dtype: int, inputs: Sequence[np.ndarray], result_f: np.ndarray) -> np.ndarray:
    """Bound of SURVEY.md §8c: |y - oracle| <= 2*gamma_{n-1}*sum|x_i| + 2*ulp_T(|oracle|)."""
    n = len(inputs)
    u = {7: 2.0 ** -24, 6: 2.0 ** -11, 9: 2.0 ** -8, 8: 2.0 ** -53, 10: 2.0 ** -4, 11: 2.0 ** -3}[dtype]
    gamma = (n - 1) * u / (1 - (n - 1) * u)
    s = np.zeros(result_f.shape, dtype=np.float64)
    for x in inputs:
        s += np.abs(to_f32(dtype, x).astype(np.float64))
    ulp = np.abs(result_f.astype(np.float64)) * (2 * u)
    return 2 * gamma * s + 2 * ulp
