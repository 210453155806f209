"""nccl_amd — Python host mirror of the MI355X tensor-bucket reduction engine.

The product is the C-ABI shared library ``nccl_amd/lib/libnccl.so`` (declared in ``include/nccl.h``,
built from ``nccl_amd/csrc``). This module binds it with ctypes and mirrors the reference's own Python
interface, nccl4py (``/root/reference/bindings/nccl4py/nccl/core/communicator.py``): ``get_unique_id``,
``Communicator.init`` / ``Communicator.init_all``, ``allreduce`` / ``reduce_scatter`` / ``allgather`` /
``reduce``, ``group()`` and ``create_pre_mul_sum``. Buffers are torch tensors on the communicator's
device (nccl4py takes CuPy/DLPack buffers); streams are HIP streams (torch.cuda streams on ROCm).

There is no fallback: if the HIP library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import dataclasses
import enum
import os
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libnccl.so")

_lib = None


class NcclError(RuntimeError):
    def __init__(self, code: int, where: str):
        self.code = code
        msg = _lib.ncclGetErrorString(code).decode() if _lib is not None else str(code)
        last = _lib.ncclGetLastError(None).decode() if _lib is not None else ""
        super().__init__(f"{where} failed: {msg} ({code}){': ' + last if last else ''}")


class Result(enum.IntEnum):  # nccl.h.in:44-53
    Success = 0
    UnhandledCudaError = 1
    SystemError = 2
    InternalError = 3
    InvalidArgument = 4
    InvalidUsage = 5
    RemoteError = 6
    InProgress = 7
    Timeout = 8


class RedOp(enum.IntEnum):  # nccl.h.in:364-372
    SUM = 0
    PROD = 1
    MAX = 2
    MIN = 3
    AVG = 4


class DataType(enum.IntEnum):  # nccl.h.in:382-395
    INT8 = 0
    UINT8 = 1
    INT32 = 2
    UINT32 = 3
    INT64 = 4
    UINT64 = 5
    FLOAT16 = 6
    FLOAT32 = 7
    FLOAT64 = 8
    BFLOAT16 = 9
    FLOAT8E4M3 = 10
    FLOAT8E5M2 = 11


SUM, PROD, MAX, MIN, AVG = RedOp.SUM, RedOp.PROD, RedOp.MAX, RedOp.MIN, RedOp.AVG
TYPE_SIZE = {0: 1, 1: 1, 2: 4, 3: 4, 4: 8, 5: 8, 6: 2, 7: 4, 8: 8, 9: 2, 10: 1, 11: 1}


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


class SimInfo(ctypes.Structure):  # ncclSimInfo_t, nccl.h.in:136-152
    _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                ("estimatedTime", ctypes.c_float)]

    @classmethod
    def default(cls) -> "SimInfo":
        s = cls()
        s.size = ctypes.sizeof(cls)
        s.magic = 0x74685283
        s.version = get_version_code_static()
        s.estimatedTime = -1.0
        return s


@dataclasses.dataclass(frozen=True)
class GroupSimInfo:
    """nccl4py GroupSimInfo (bindings/nccl4py/nccl/core/group.py:28-36)."""
    estimated_time: float  # seconds


class MemStat(enum.IntEnum):  # ncclCommMemStat_t, nccl.h.in:333-338
    GPU_MEM_SUSPEND = 0
    GPU_MEM_SUSPENDED = 1
    GPU_MEM_PERSIST = 2
    GPU_MEM_TOTAL = 3


class Config(ctypes.Structure):  # ncclConfig_t, nccl.h.in:84-108
    _fields_ = [
        ("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
        ("blocking", ctypes.c_int), ("cgaClusterSize", ctypes.c_int), ("minCTAs", ctypes.c_int),
        ("maxCTAs", ctypes.c_int), ("netName", ctypes.c_char_p), ("splitShare", ctypes.c_int),
        ("trafficClass", ctypes.c_int), ("commName", ctypes.c_char_p), ("collnetEnable", ctypes.c_int),
        ("CTAPolicy", ctypes.c_int), ("shrinkShare", ctypes.c_int), ("nvlsCTAs", ctypes.c_int),
        ("nChannelsPerNetPeer", ctypes.c_int), ("nvlinkCentricSched", ctypes.c_int),
        ("graphUsageMode", ctypes.c_int), ("numRmaCtx", ctypes.c_int), ("maxP2pPeers", ctypes.c_int),
        ("graphStreamOrdering", ctypes.c_int),
    ]

    @classmethod
    def default(cls, **kw) -> "Config":
        undef = -(2 ** 31)
        c = cls()
        c.size = ctypes.sizeof(cls)
        c.magic = 0xCAFEBEEF
        c.version = get_version_code_static()
        for name, ty in cls._fields_[3:]:
            setattr(c, name, None if ty is ctypes.c_char_p else undef)
        for k, v in kw.items():
            setattr(c, k, v.encode() if isinstance(v, str) else v)
        return c


def get_version_code_static() -> int:
    return 2 * 10000 + 30 * 100 + 7  # NCCL_VERSION(2,30,7)


# Every function include/nccl.h declares (the C-ABI surface the tests check for).
EXPORTED = [
    "ncclMemAlloc", "ncclMemFree", "ncclGetVersion", "ncclGetUniqueId", "ncclCommInitRankConfig",
    "ncclCommInitRank", "ncclCommInitAll", "ncclCommFinalize", "ncclCommDestroy", "ncclCommAbort",
    "ncclGetErrorString", "ncclGetLastError", "ncclCommGetAsyncError", "ncclCommCount", "ncclCommCuDevice",
    "ncclCommUserRank", "ncclRedOpCreatePreMulSum", "ncclRedOpDestroy", "ncclReduce", "ncclAllReduce",
    "ncclReduceScatter", "ncclAllGather", "ncclGroupStart", "ncclGroupEnd",
    "ncclCommRegister", "ncclCommDeregister", "ncclCommWindowRegister", "ncclCommWindowDeregister",
    "ncclWinGetUserPtr", "ncclCommInitRankScalable", "ncclCommMemStats", "ncclGroupSimulateEnd",
]


WIN_DEFAULT = 0x00          # nccl.h.in:64-68
WIN_COLL_SYMMETRIC = 0x01
WIN_STRICT_ORDERING = 0x02
WIN_REQUIRED_ALIGNMENT = 4096


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libnccl.so (RTLD_LOCAL; the library is linked -Bsymbolic so RCCL, which torch loads, can
    never interpose on its internal calls)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64 (same soname as /opt/rocm's). If this
    # library were loaded first it would pull in /opt/rocm's runtime and torch would later bring a second
    # one ("no ROCm-capable device" from whichever initialises second), so let torch load its runtime first
    # and bind to that one.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    p = path or os.environ.get("NCCL_AMD_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise RuntimeError(f"nccl_amd: HIP library {p} is missing — build it first (make, or __graft_entry__.build())")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
    R, P, I, S, U64 = ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64
    sig = {
        "ncclGetVersion": (R, [ctypes.POINTER(I)]),
        "ncclGetUniqueId": (R, [ctypes.POINTER(UniqueId)]),
        "ncclCommInitRank": (R, [ctypes.POINTER(P), I, UniqueId, I]),
        "ncclCommInitRankConfig": (R, [ctypes.POINTER(P), I, UniqueId, I, ctypes.POINTER(Config)]),
        "ncclCommInitAll": (R, [ctypes.POINTER(P), I, ctypes.POINTER(I)]),
        "ncclCommFinalize": (R, [P]),
        "ncclCommDestroy": (R, [P]),
        "ncclCommAbort": (R, [P]),
        "ncclGetErrorString": (ctypes.c_char_p, [I]),
        "ncclGetLastError": (ctypes.c_char_p, [P]),
        "ncclCommGetAsyncError": (R, [P, ctypes.POINTER(I)]),
        "ncclCommCount": (R, [P, ctypes.POINTER(I)]),
        "ncclCommCuDevice": (R, [P, ctypes.POINTER(I)]),
        "ncclCommUserRank": (R, [P, ctypes.POINTER(I)]),
        "ncclRedOpCreatePreMulSum": (R, [ctypes.POINTER(I), P, I, I, P]),
        "ncclRedOpDestroy": (R, [I, P]),
        "ncclAllReduce": (R, [P, P, S, I, I, P, P]),
        "ncclReduceScatter": (R, [P, P, S, I, I, P, P]),
        "ncclAllGather": (R, [P, P, S, I, P, P]),
        "ncclReduce": (R, [P, P, S, I, I, I, P, P]),
        "ncclGroupStart": (R, []),
        "ncclGroupEnd": (R, []),
        "ncclMemAlloc": (R, [ctypes.POINTER(P), S]),
        "ncclCommRegister": (R, [P, P, S, ctypes.POINTER(P)]),
        "ncclCommDeregister": (R, [P, P]),
        "ncclCommWindowRegister": (R, [P, P, S, ctypes.POINTER(P), I]),
        "ncclCommWindowDeregister": (R, [P, P]),
        "ncclWinGetUserPtr": (R, [P, P, ctypes.POINTER(P)]),
        "ncclMemFree": (R, [P]),
        "ncclCommInitRankScalable": (R, [ctypes.POINTER(P), I, I, I, ctypes.POINTER(UniqueId), ctypes.POINTER(Config)]),
        "ncclCommMemStats": (R, [P, I, ctypes.POINTER(U64)]),
        "ncclGroupSimulateEnd": (R, [ctypes.POINTER(SimInfo)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def _check(code: int, where: str) -> None:
    if code != 0:
        raise NcclError(code, where)


def get_version() -> int:
    v = ctypes.c_int()
    _check(load().ncclGetVersion(ctypes.byref(v)), "ncclGetVersion")
    return v.value


def get_unique_id() -> bytes:
    uid = UniqueId()
    _check(load().ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
    return ctypes.string_at(ctypes.addressof(uid), 128)


def _uid(b: bytes) -> UniqueId:
    u = UniqueId()
    ctypes.memmove(ctypes.byref(u), b, 128)
    return u


def group_start() -> None:
    _check(load().ncclGroupStart(), "ncclGroupStart")


def group_end(*, simulate: bool = False) -> Optional[GroupSimInfo]:
    """nccl4py group_end (group.py:54-76): simulate=True plans the group's collectives without launching
    them (ncclGroupSimulateEnd) and returns the cost model's estimate, in seconds."""
    if not simulate:
        _check(load().ncclGroupEnd(), "ncclGroupEnd")
        return None
    si = SimInfo.default()
    _check(load().ncclGroupSimulateEnd(ctypes.byref(si)), "ncclGroupSimulateEnd")
    return GroupSimInfo(estimated_time=si.estimatedTime * 1e-6)


@contextlib.contextmanager
def group():
    group_start()
    try:
        yield
    finally:
        group_end()


def torch_dtype_to_nccl(dtype) -> int:
    import torch
    m = {
        torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
        torch.float64: 8, torch.bfloat16: 9,
    }
    for name, code in (("uint32", 3), ("uint64", 5), ("float8_e4m3fn", 10), ("float8_e5m2", 11)):
        if hasattr(torch, name):
            m[getattr(torch, name)] = code
    if dtype not in m:
        raise TypeError(f"unsupported dtype {dtype}")
    return m[dtype]


def _stream_ptr(stream, device: int) -> int:
    import torch
    if stream is None:
        return torch.cuda.current_stream(device).cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


_HIP = None


def dedicated_stream(device: int = 0):
    """A torch ExternalStream with a hardware queue of its own (created with a full CU mask).

    Only needed when several ranks share one GPU inside one process AND the caller replays captured
    graphs of their collectives on its own streams: HIP multiplexes a process's streams onto a few
    hardware queues, and two ranks' kernels on one queue would serialise (each spins on the other).
    Direct ncclAllReduce/... calls handle this inside the library (ncclComm::internalStream)."""
    global _HIP
    import torch
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    ncu = torch.cuda.get_device_properties(device).multi_processor_count
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)(*([0xFFFFFFFF] * words))
    if ncu % 32:
        mask[words - 1] = (1 << (ncu % 32)) - 1
    s = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = _HIP.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
    return torch.cuda.ExternalStream(s.value, device=device)


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


class Window:
    """An ncclWindow_t; the handle storage stays alive until the (possibly deferred) registration ends."""

    def __init__(self, comm: "Communicator"):
        self.comm = comm
        self._h = ctypes.c_void_p()

    @property
    def handle(self) -> int:
        return self._h.value or 0


class Communicator:
    """Mirror of nccl4py's Communicator (bindings/nccl4py/nccl/core/communicator.py:223)."""

    def __init__(self, ptr: int):
        self._comm = ptr
        self._nranks = None
        self._rank = None
        self._device = None

    # ---- construction (nccl4py Communicator.init / init_all) ----
    @classmethod
    def init(cls, nranks: int, rank: int, unique_id, config: Optional[Config] = None) -> "Communicator":
        """unique_id: one id (bytes), or a sequence of ids for ncclCommInitRankScalable (nccl4py
        communicator.py:333-334)."""
        lib = load()
        c = ctypes.c_void_p()
        if not isinstance(unique_id, (bytes, bytearray)):
            ids = list(unique_id)
            arr = (UniqueId * len(ids))(*[_uid(b) for b in ids])
            rc = lib.ncclCommInitRankScalable(ctypes.byref(c), nranks, rank, len(ids), arr,
                                              ctypes.byref(config) if config is not None else None)
            if not (rc == Result.InProgress and config is not None and config.blocking == 0):
                _check(rc, "ncclCommInitRankScalable")
            return cls(c.value)
        if config is None:
            _check(lib.ncclCommInitRank(ctypes.byref(c), nranks, _uid(unique_id), rank), "ncclCommInitRank")
        else:
            rc = lib.ncclCommInitRankConfig(ctypes.byref(c), nranks, _uid(unique_id), rank, ctypes.byref(config))
            if not (rc == Result.InProgress and config.blocking == 0):  # non-blocking: poll wait_ready()
                _check(rc, "ncclCommInitRankConfig")
        return cls(c.value)

    def wait_ready(self, timeout_s: float = 600.0) -> None:
        """Non-blocking communicators: poll ncclCommGetAsyncError until it leaves ncclInProgress."""
        import time
        t0 = time.time()
        while True:
            e = self.async_error()
            if e != Result.InProgress:
                _check(e, "ncclCommInitRankConfig (non-blocking)")
                return
            if time.time() - t0 > timeout_s:
                raise TimeoutError("communicator still initialising")
            time.sleep(0.001)

    @classmethod
    def init_all(cls, devices: Sequence[int] | int) -> list["Communicator"]:
        lib = load()
        devs = list(range(devices)) if isinstance(devices, int) else list(devices)
        arr = (ctypes.c_void_p * len(devs))()
        dl = (ctypes.c_int * len(devs))(*devs)
        _check(lib.ncclCommInitAll(arr, len(devs), dl), "ncclCommInitAll")
        return [cls(arr[i]) for i in range(len(devs))]

    # ---- properties ----
    @property
    def ptr(self) -> int:
        return self._comm

    @property
    def nranks(self) -> int:
        if self._nranks is None:
            v = ctypes.c_int()
            _check(load().ncclCommCount(self._comm, ctypes.byref(v)), "ncclCommCount")
            self._nranks = v.value
        return self._nranks

    @property
    def rank(self) -> int:
        if self._rank is None:
            v = ctypes.c_int()
            _check(load().ncclCommUserRank(self._comm, ctypes.byref(v)), "ncclCommUserRank")
            self._rank = v.value
        return self._rank

    @property
    def device(self) -> int:
        if self._device is None:
            v = ctypes.c_int()
            _check(load().ncclCommCuDevice(self._comm, ctypes.byref(v)), "ncclCommCuDevice")
            self._device = v.value
        return self._device

    def mem_stats(self, stat: "MemStat" = MemStat.GPU_MEM_TOTAL) -> int:
        """ncclCommMemStats: device bytes this communicator holds (everything is persistent here)."""
        v = ctypes.c_uint64()
        _check(load().ncclCommMemStats(self._comm, int(stat), ctypes.byref(v)), "ncclCommMemStats")
        return v.value

    def async_error(self) -> int:
        v = ctypes.c_int()
        _check(load().ncclCommGetAsyncError(self._comm, ctypes.byref(v)), "ncclCommGetAsyncError")
        return v.value

    # ---- collectives on torch tensors ----
    def _check_tensors(self, where: str, *ts) -> None:
        """Buffers handed to the C ABI are raw pointers: they must be dense and on this communicator's GPU."""
        for t in ts:
            if t is None:
                continue
            if not t.is_contiguous():
                raise ValueError(f"{where}: tensors must be contiguous")
            if t.device.type != "cuda" or t.device.index != self.device:
                raise ValueError(f"{where}: tensor on {t.device}, communicator on cuda:{self.device}")

    def allreduce(self, sendbuf, recvbuf, op=RedOp.SUM, *, stream=None) -> None:
        self._check_tensors("allreduce", sendbuf, recvbuf)
        if sendbuf.numel() != recvbuf.numel() or sendbuf.dtype != recvbuf.dtype:
            raise ValueError("allreduce: sendbuf/recvbuf must match in dtype and count")
        self.all_reduce_raw(sendbuf.data_ptr(), recvbuf.data_ptr(), sendbuf.numel(),
                            torch_dtype_to_nccl(sendbuf.dtype), int(op), _stream_ptr(stream, self.device))

    def reduce_scatter(self, sendbuf, recvbuf, op=RedOp.SUM, *, stream=None) -> None:
        self._check_tensors("reduce_scatter", sendbuf, recvbuf)
        if sendbuf.numel() != recvbuf.numel() * self.nranks or sendbuf.dtype != recvbuf.dtype:
            raise ValueError("reduce_scatter: sendbuf must hold nranks * recvbuf.numel() elements of the same dtype")
        self.reduce_scatter_raw(sendbuf.data_ptr(), recvbuf.data_ptr(), recvbuf.numel(),
                                torch_dtype_to_nccl(sendbuf.dtype), int(op), _stream_ptr(stream, self.device))

    def allgather(self, sendbuf, recvbuf, *, stream=None) -> None:
        self._check_tensors("allgather", sendbuf, recvbuf)
        if recvbuf.numel() != sendbuf.numel() * self.nranks or sendbuf.dtype != recvbuf.dtype:
            raise ValueError("allgather: recvbuf must hold nranks * sendbuf.numel() elements of the same dtype")
        self.all_gather_raw(sendbuf.data_ptr(), recvbuf.data_ptr(), sendbuf.numel(),
                            torch_dtype_to_nccl(sendbuf.dtype), _stream_ptr(stream, self.device))

    def reduce(self, sendbuf, recvbuf, op=RedOp.SUM, root: int = 0, *, stream=None) -> None:
        self._check_tensors("reduce", sendbuf, recvbuf if self.rank == root else None)
        if self.rank == root and (recvbuf is None or recvbuf.numel() != sendbuf.numel()
                                  or recvbuf.dtype != sendbuf.dtype):
            raise ValueError("reduce: the root's recvbuf must match sendbuf in dtype and count")
        self.reduce_raw(sendbuf.data_ptr(), _ptr(recvbuf), sendbuf.numel(), torch_dtype_to_nccl(sendbuf.dtype),
                        int(op), root, _stream_ptr(stream, self.device))

    # ---- collectives on raw device pointers (the C ABI one-to-one) ----
    def all_reduce_raw(self, send: int, recv: int, count: int, dtype: int, op: int, stream: int) -> None:
        _check(load().ncclAllReduce(send, recv, count, dtype, op, self._comm, stream), "ncclAllReduce")

    def reduce_scatter_raw(self, send: int, recv: int, recvcount: int, dtype: int, op: int, stream: int) -> None:
        _check(load().ncclReduceScatter(send, recv, recvcount, dtype, op, self._comm, stream), "ncclReduceScatter")

    def all_gather_raw(self, send: int, recv: int, sendcount: int, dtype: int, stream: int) -> None:
        _check(load().ncclAllGather(send, recv, sendcount, dtype, self._comm, stream), "ncclAllGather")

    def reduce_raw(self, send: int, recv: Optional[int], count: int, dtype: int, op: int, root: int,
                   stream: int) -> None:
        _check(load().ncclReduce(send, recv, count, dtype, op, root, self._comm, stream), "ncclReduce")

    # ---- registration (nccl.h.in:301-360; nccl4py Communicator.register_buffer / register_window) ----
    def register_buffer(self, ptr: int, size: int) -> int:
        """ncclCommRegister (local); returns the handle."""
        h = ctypes.c_void_p()
        _check(load().ncclCommRegister(self._comm, ptr, size, ctypes.byref(h)), "ncclCommRegister")
        return h.value or 0

    def deregister_buffer(self, handle: int) -> None:
        _check(load().ncclCommDeregister(self._comm, handle), "ncclCommDeregister")

    def register_window(self, ptr: int, size: int, flags: int = WIN_COLL_SYMMETRIC) -> "Window":
        """ncclCommWindowRegister (collective: every rank calls it; one thread driving several ranks
        calls it inside group(), and the handle is filled in when the group ends)."""
        w = Window(self)
        _check(load().ncclCommWindowRegister(self._comm, ptr, size, ctypes.byref(w._h), flags),
               "ncclCommWindowRegister")
        return w

    def deregister_window(self, win) -> None:
        h = win.handle if isinstance(win, Window) else win
        _check(load().ncclCommWindowDeregister(self._comm, h), "ncclCommWindowDeregister")

    def window_user_ptr(self, win) -> int:
        h = win.handle if isinstance(win, Window) else win
        p = ctypes.c_void_p()
        _check(load().ncclWinGetUserPtr(self._comm, h, ctypes.byref(p)), "ncclWinGetUserPtr")
        return p.value or 0

    # ---- custom operators ----
    def create_pre_mul_sum(self, scalar, dtype: int, device_scalar_ptr: Optional[int] = None) -> int:
        """ncclRedOpCreatePreMulSum; `scalar` is a host value (ncclScalarHostImmediate) unless
        `device_scalar_ptr` is given (ncclScalarDevice)."""
        import numpy as np
        op = ctypes.c_int()
        if device_scalar_ptr is not None:
            _check(load().ncclRedOpCreatePreMulSum(ctypes.byref(op), device_scalar_ptr, dtype, 0, self._comm),
                   "ncclRedOpCreatePreMulSum")
        else:
            npdt = {0: np.int8, 1: np.uint8, 2: np.int32, 3: np.uint32, 4: np.int64, 5: np.uint64, 6: np.float16,
                    7: np.float32, 8: np.float64}.get(dtype)
            if npdt is not None:
                buf = np.array([scalar], dtype=npdt).tobytes()
            else:  # bf16 / fp8: caller passes the raw bit pattern as an int
                buf = int(scalar).to_bytes(TYPE_SIZE[dtype], "little")
            cbuf = ctypes.create_string_buffer(buf, 8)
            _check(load().ncclRedOpCreatePreMulSum(ctypes.byref(op), cbuf, dtype, 1, self._comm),
                   "ncclRedOpCreatePreMulSum")
        return op.value

    def destroy_op(self, op: int) -> None:
        _check(load().ncclRedOpDestroy(op, self._comm), "ncclRedOpDestroy")

    # ---- teardown ----
    def finalize(self) -> None:
        _check(load().ncclCommFinalize(self._comm), "ncclCommFinalize")

    def destroy(self) -> None:
        if self._comm:
            _check(load().ncclCommDestroy(self._comm), "ncclCommDestroy")
            self._comm = 0

    def abort(self) -> None:
        if self._comm:
            _check(load().ncclCommAbort(self._comm), "ncclCommAbort")
            self._comm = 0


def ddp_comm_hook(comm: "Communicator"):
    """A torch DDP communication hook that reduces every gradient bucket with this engine (ncclAvg, in
    place, on the current stream) instead of the process group's backend:
    ``ddp_model.register_comm_hook(None, nccl_amd.ddp_comm_hook(comm))``."""
    import torch

    def hook(state, bucket):
        t = bucket.buffer()
        comm.allreduce(t, t, RedOp.AVG)
        fut = torch.futures.Future()
        fut.set_result(t)
        return fut

    return hook
