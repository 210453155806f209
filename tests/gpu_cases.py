"""Shared helpers for the GPU parity tests: run a collective through the C ABI (nccl_amd) on torch
device buffers and compare with the CPU oracle. Imported by tests only."""
from __future__ import annotations

import os

import numpy as np

import oracle

# dtype code -> torch dtype name used to allocate raw storage of the same width
TORCH_STORAGE = {0: "int8", 1: "uint8", 2: "int32", 3: "int32", 4: "int64", 5: "int64", 6: "int16", 7: "float32",
                 8: "float64", 9: "int16", 10: "uint8", 11: "uint8"}
FLOAT_TYPES = {6, 7, 8, 9, 10, 11}


def to_device(arr: np.ndarray, device, offset_elems: int = 0):
    """Copy a numpy storage array to a fresh device buffer (device "pinned": pinned host memory, which the kernels
    reach across PCIe); `offset_elems` > 0 returns a view that is deliberately NOT 16-byte aligned (exercises the
    reference's unaligned fallback)."""
    import torch
    raw = np.ascontiguousarray(arr).view(np.uint8)
    es = arr.dtype.itemsize
    if device == "pinned":
        buf = torch.empty(raw.size + offset_elems * es + 64, dtype=torch.uint8, pin_memory=True)
    else:
        buf = torch.empty(raw.size + offset_elems * es + 64, dtype=torch.uint8, device=device)
    view = buf[offset_elems * es: offset_elems * es + raw.size]
    view.copy_(torch.from_numpy(raw.copy()))
    return buf, view


def from_device(view, dtype_np) -> np.ndarray:
    return view.cpu().numpy().view(dtype_np).copy()


def _raw(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a).view({1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize])


def same_bits(a: np.ndarray, b: np.ndarray, dtype: int) -> bool:
    """Bitwise equality of every element — the sign of zero included (+0 and -0 differ) — except NaN payloads: a
    float NaN must sit where the oracle has one, its sign and payload are not compared here. (A NaN generated from
    non-NaN inputs, or two NaNs meeting, is the hardware's: x86 and gfx950 default NaNs differ in sign. The single-NaN
    case is compared bit for bit by test_gpu_collectives.py::test_single_nan_payloads)"""
    if a.shape != b.shape:
        return False
    ua, ub = _raw(a), _raw(b)
    if dtype not in FLOAT_TYPES:
        return np.array_equal(ua, ub)
    na, nb = np.isnan(oracle.to_f32(dtype, a)), np.isnan(oracle.to_f32(dtype, b))
    return bool(np.array_equal(na, nb) and np.array_equal(ua[~na], ub[~na]))


def make_inputs(n: int, dtype: int, count: int, seed: int, kind: int = 0):
    return [oracle.fill(dtype, seed * 131 + r, count, kind) for r in range(n)]


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def ring_channels(n: int, ranks_per_gpu: int | None = None) -> int:
    """The channel count K a NCCL_ALGO=RING / NCCL_AMD_REF_ORDER AllReduce is planned on (enqueue.cc
    refChannelCount): NCCL_AMD_REF_NCHANNELS when set, else the communicator's co-resident channel cap —
    NCCL_MAX_CTAS / NCCL_MAX_NCHANNELS (default 256) capped at 2 workgroups per CU for one rank per GPU, at CUs
    divided by the ranks per GPU when they share one (enqueue.cc coResidentChannelCap; every test rank shares the box's
    one GPU) — and at most the reference's MAXCHANNELS = 64 (src/include/device.h:91) and the channel cap."""
    import torch
    cap = _env_int("NCCL_MAX_CTAS", _env_int("NCCL_MAX_NCHANNELS", 256))
    cap = max(1, min(cap, 256))
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rpg = ranks_per_gpu or n
    cap = max(1, min(cap, 2 * cus if rpg == 1 else cus // rpg))
    k = _env_int("NCCL_AMD_REF_NCHANNELS", 0) or cap
    return max(1, min(k, 64, cap))  # every part needs a workgroup: never more parts than the channel cap


def ring_runs(n: int) -> bool:
    """Whether NCCL_ALGO=RING (from the environment the communicator was created under) runs the ring kernel for
    an AllReduce: two staging slots are needed (enqueue.cc planColl). NCCL_PROTO naming LL or LL128 alone runs the
    ring on that protocol's partition (ref_proto); with several LL-class protocols and no Simple the LL kernel
    takes what fits its line area and the ring the rest, a size rule this helper does not restate: the tests
    never use that combination with NCCL_ALGO=RING (ValueError)."""
    if os.environ.get("NCCL_ALGO", "").upper() != "RING" or n < 2:
        return False
    proto = os.environ.get("NCCL_PROTO", "")
    if proto:
        toks = {t.strip().lower() for t in proto.lstrip("^").split(",")}
        simple = ("simple" not in toks) if proto.startswith("^") else ("simple" in toks)
        if not simple and ref_proto()[0] == oracle.PROTO_SIMPLE:
            raise ValueError(f"NCCL_ALGO=RING with NCCL_PROTO={proto}: the AllReduce order depends on the LL capacity")
    return _env_int("NCCL_AMD_NSLOTS", 2) >= 2


def ref_order_runs(n: int) -> bool:
    """Whether NCCL_AMD_REF_ORDER=1 (from the communicator's environment) puts AllReduce on the reference's ring
    partition (the direct kernel in that order; enqueue.cc planColl): any size and protocol, unless
    NCCL_ALGO=TREE / RING takes the reference's own chain / ring instead."""
    return n >= 2 and _env_int("NCCL_AMD_REF_ORDER", 0) != 0 and \
        os.environ.get("NCCL_ALGO", "").upper() not in ("TREE", "RING")


def ref_proto() -> tuple[int, int]:
    """The protocol whose ring partition NCCL_AMD_REF_ORDER walks and that protocol's buffer size (0 = default):
    LL or LL128 when NCCL_PROTO enables that one protocol alone, Simple otherwise (enqueue.cc loadTuning)."""
    proto = os.environ.get("NCCL_PROTO", "")
    on = {"ll": True, "simple": True, "ll128": _env_int("NCCL_AMD_LL128", 0) != 0}
    if proto:
        excl = proto.startswith("^")
        toks = {t.strip().lower() for t in proto.lstrip("^").split(",")}
        on = {k: ((k not in toks) and (on[k] if k == "ll128" else True)) if excl else (k in toks) for k in on}
        if excl and not on["ll"] and not on["simple"] and "ll128" not in toks:
            on["ll128"] = True  # LL128 at its gate is on when it is the only protocol left (enqueue.cc resolveFuncTuning)
    if on["ll"] and not on["simple"] and not on["ll128"]:
        return oracle.PROTO_LL, _env_int("NCCL_LL_BUFFSIZE", 0)
    if on["ll128"] and not on["ll"] and not on["simple"]:
        return oracle.PROTO_LL128, _env_int("NCCL_LL128_BUFFSIZE", 0)
    return oracle.PROTO_SIMPLE, _env_int("NCCL_BUFFSIZE", 0)


def expected(coll: str, inputs, dtype: int, op: int, root: int = 0, algo: str = ""):
    if coll == "allreduce":
        # NCCL_ALGO=TREE folds every element in the chain's order; NCCL_ALGO=RING in the reference's ring order
        # over its own channel parts and loops (NCCL_MAX_CTAS / NCCL_BUFFSIZE as set for the communicator);
        # every other path in the one-loop ring order
        n = len(inputs)
        algo = algo or os.environ.get("NCCL_ALGO", "").upper()
        if algo == "TREE":
            out = oracle.all_reduce_chain(inputs, dtype, op)
        elif (algo == "RING" and ring_runs(n)) or ref_order_runs(n):
            proto, buff = ref_proto()
            out = oracle.all_reduce_ring_nccl(inputs, dtype, op, ring_channels(n), buff, proto)
        else:
            out = oracle.all_reduce(inputs, dtype, op)
        return [out] * len(inputs)
    if coll == "reducescatter":
        return oracle.reduce_scatter(inputs, dtype, op)
    if coll == "allgather":
        out = oracle.all_gather(inputs)
        return [out] * len(inputs)
    if coll == "reduce":
        return [oracle.reduce(inputs, dtype, op, root)]
    raise ValueError(coll)


def out_count(coll: str, n: int, count: int) -> int:
    return {"allreduce": count, "reducescatter": count // n, "allgather": count * n, "reduce": count}[coll]


def launch(comm, coll: str, send_view, recv_view, count: int, dtype: int, op: int, root: int, stream_ptr: int):
    n = comm.nranks
    if coll == "allreduce":
        comm.all_reduce_raw(send_view.data_ptr(), recv_view.data_ptr(), count, dtype, op, stream_ptr)
    elif coll == "reducescatter":
        comm.reduce_scatter_raw(send_view.data_ptr(), recv_view.data_ptr(), count // n, dtype, op, stream_ptr)
    elif coll == "allgather":
        comm.all_gather_raw(send_view.data_ptr(), recv_view.data_ptr(), count, dtype, stream_ptr)
    elif coll == "reduce":
        rp = recv_view.data_ptr() if recv_view is not None else None
        comm.reduce_raw(send_view.data_ptr(), rp, count, dtype, op, root, stream_ptr)


# A compact but broad case list: (collective, dtype, op, count, misalign)
def case_list(n: int, quick: bool = False):
    cases = []
    counts = [1, 5, 4096 + 3, 300_001] if not quick else [5, 70_001]
    for coll in ("allreduce", "reducescatter", "allgather", "reduce"):
        for dtype in (7, 9, 6, 2, 3, 4, 0, 1, 5, 8, 10, 11):
            ops = [0] if coll == "allgather" else [0, 1, 2, 3, 4]
            for op in ops:
                if quick and dtype not in (7, 9, 2) and op != 0:
                    continue
                for count in counts:
                    if coll == "reducescatter":
                        count = max(1, count // n) * n
                    cases.append((coll, dtype, op, count, 0))
        cases.append((coll, 7, 0, 100_003 * n, 1))   # misaligned base pointers
        cases.append((coll, 9, 0, 10_001 * n, 3))
    return cases


def run_case(comms_and_streams, coll, dtype, op, count, misalign, seed, inplace=False, root=0, sync=True,
             inputs=None, algo="", host=False):
    """Run one collective on every (comm, stream) of this process; returns list of error strings.
    `comms_and_streams` holds the ranks owned by this process: [(comm, torch stream), ...]; the
    inputs of ALL ranks are regenerated deterministically so each process can check its own ranks.
    `host` (a bool, or one per rank): that rank's buffers are pinned host memory."""
    import torch
    n = comms_and_streams[0][0].nranks
    if inputs is None:
        inputs = make_inputs(n, dtype, count, seed)
    exp = expected(coll, inputs, dtype, op, root, algo)
    npdt = oracle.NP_STORAGE[dtype]
    es = np.dtype(npdt).itemsize
    ocount = out_count(coll, n, count)
    keep, views = [], []
    per_rank = misalign if isinstance(misalign, (list, tuple)) else None
    for comm, stream in comms_and_streams:
        r = comm.rank
        if per_rank is not None:  # each rank's buffers misaligned differently (protocol choice must not care)
            misalign = per_rank[r % len(per_rank)]
        dev = torch.device("cuda", comm.device)
        on_host = host[r % len(host)] if isinstance(host, (list, tuple)) else host
        with torch.cuda.device(dev):
            if on_host:
                dev = "pinned"
            if inplace:
                # one buffer: AR send==recv; RS recv = send + r*recvcount; AG send = recv + r*sendcount
                if coll in ("allreduce", "reduce"):
                    buf, sv = to_device(inputs[r], dev, misalign)
                    rv = sv
                elif coll == "reducescatter":
                    buf, sv = to_device(inputs[r], dev, misalign)
                    rc = count // n
                    rv = sv[r * rc * es:(r + 1) * rc * es]
                else:  # allgather
                    full = np.zeros(count * n, dtype=npdt)
                    full[r * count:(r + 1) * count] = inputs[r]
                    buf, rv = to_device(full, dev, misalign)
                    sv = rv[r * count * es:(r + 1) * count * es]
                keep.append(buf)
            else:
                b1, sv = to_device(inputs[r], dev, misalign)
                rv = None
                if coll != "reduce" or r == root:
                    b2, rv = to_device(np.zeros(ocount, dtype=npdt), dev, misalign)
                    keep.append(b2)
                keep.append(b1)
            views.append((comm, stream, sv, rv))
    import nccl_amd
    torch.cuda.synchronize()
    with nccl_amd.group():
        for comm, stream, sv, rv in views:
            launch(comm, coll, sv, rv, count, dtype, op, root, stream.cuda_stream)
    errs = []
    for comm, stream, sv, rv in views:
        stream.synchronize()
        ae = comm.async_error()
        if ae != 0:
            errs.append(f"rank {comm.rank}: async error {ae}")
            continue
        r = comm.rank
        if coll == "reduce" and r != root:
            continue
        got = from_device(rv, npdt)
        want = exp[0] if coll == "reduce" else exp[r]
        if not same_bits(got, want, dtype):
            bad = np.nonzero(got != want)[0]
            errs.append(f"rank {r} {coll} dt={dtype} op={op} count={count} mis={misalign} inplace={inplace}: "
                        f"{bad.size} mismatches, first at {bad[:5].tolist()} got {got[bad[:3]].tolist()} "
                        f"want {want[bad[:3]].tolist()}")
    return errs


def run_group(comms_and_streams, ops, seed):
    """Several collectives [(coll, dtype, op, count), ...] issued inside ONE group (so consecutive ops that plan
    onto the same kernel are batched into one launch), out of place, checked bit-exactly; returns errors."""
    import torch
    import nccl_amd
    n = comms_and_streams[0][0].nranks
    plan = []
    for k, (coll, dtype, op, count) in enumerate(ops):
        inputs = make_inputs(n, dtype, count, seed * 100 + k)
        exp = expected(coll, inputs, dtype, op, 0)
        npdt = oracle.NP_STORAGE[dtype]
        bufs = {}
        for comm, _ in comms_and_streams:
            dev = torch.device("cuda", comm.device)
            b1, sv = to_device(inputs[comm.rank], dev, 0)
            b2, rv = to_device(np.zeros(out_count(coll, n, count), dtype=npdt), dev, 0)
            bufs[comm.rank] = (b1, sv, b2, rv)
        plan.append((coll, dtype, op, count, exp, npdt, bufs))
    torch.cuda.synchronize()
    with nccl_amd.group():
        for coll, dtype, op, count, _, _, bufs in plan:
            for comm, stream in comms_and_streams:
                _, sv, _, rv = bufs[comm.rank]
                launch(comm, coll, sv, rv, count, dtype, op, 0, stream.cuda_stream)
    errs = []
    for comm, stream in comms_and_streams:
        stream.synchronize()
        if comm.async_error():
            errs.append(f"rank {comm.rank}: async error {comm.async_error()}")
    for k, (coll, dtype, op, count, exp, npdt, bufs) in enumerate(plan):
        for comm, _ in comms_and_streams:
            if coll == "reduce" and comm.rank != 0:
                continue
            got = from_device(bufs[comm.rank][3], npdt)
            want = exp[0] if coll == "reduce" else exp[comm.rank]
            if not same_bits(got, want, dtype):
                bad = np.nonzero(got != want)[0]
                errs.append(f"group op {k} rank {comm.rank} {coll} dt={dtype} op={op} count={count}: "
                            f"{bad.size} mismatches, first at {bad[:5].tolist()}")
    return errs
