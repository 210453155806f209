"""The eager-registration churn pattern without the library, on the HIP runtime a PyTorch process binds (torch's
bundled libamdhip64): two processes on one GPU, each iteration allocating a send / receive pair through PyTorch's
caching allocator (same ranges every time), exporting both as dma-bufs (hipMemGetHandleForAddressRange, as
register.cc regCreate), handing the fds to the peer over a UNIX socket, mapping the peer's (hipImportExternalMemory +
hipExternalMemoryGetMappedBuffer, as ipc.cc importFd), freeing its own pair, and unmapping the peer's (hipFree +
hipDestroyExternalMemory + close, as ipc.cc releaseLocked) at once (UNMAP=now), one iteration later (late) or never.
No kernel touches the mappings. Counts exports that fail, and retries them RETRY times 1 ms apart.

  python3 scripts/eager_churn_probe.py [ITERS=8] [UNMAP=now|late|never] [RETRY=0]     one JSON line per rank
"""
import ctypes
import json
import multiprocessing as mp
import os
import socket
import sys
import time

MIB = 1 << 20


class HandleDesc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("pad", ctypes.c_int), ("fd_or_ptr", ctypes.c_uint64), ("name", ctypes.c_uint64),
                ("size", ctypes.c_ulonglong), ("flags", ctypes.c_uint), ("reserved", ctypes.c_uint * 16)]


class BufferDesc(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_ulonglong), ("size", ctypes.c_ulonglong), ("flags", ctypes.c_uint),
                ("reserved", ctypes.c_uint * 16)]


def worker(rank, iters, unmap, retry, q):
    import torch
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so")
    name = b"\0eager_churn_probe_%d" % os.getppid()
    if rank == 0:
        srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        srv.bind(name)
        srv.listen(1)
        s, _ = srv.accept()
    else:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        for _ in range(200):
            try:
                s.connect(name)
                break
            except OSError:
                time.sleep(0.05)

    def export(t):
        base, size = ctypes.c_void_p(), ctypes.c_size_t()
        assert hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(t.data_ptr())) == 0
        fd = ctypes.c_int(-1)
        for attempt in range(retry + 1):
            rc = hip.hipMemGetHandleForAddressRange(ctypes.byref(fd), base, size, 1, ctypes.c_ulonglong(0))
            if rc == 0:
                return fd.value, size.value, attempt, base.value
            hip.hipGetLastError()
            time.sleep(0.001)
        return -1, size.value, retry + 1, base.value

    def imp(fd, size):
        hd = HandleDesc()
        hd.type = 1
        hd.fd_or_ptr = fd
        hd.size = size
        em = ctypes.c_void_p()
        assert hip.hipImportExternalMemory(ctypes.byref(em), ctypes.byref(hd)) == 0
        bd = BufferDesc()
        bd.size = size
        p = ctypes.c_void_p()
        assert hip.hipExternalMemoryGetMappedBuffer(ctypes.byref(p), em, ctypes.byref(bd)) == 0
        return (p, em, fd)

    def unmap_all(maps):
        for p, em, fd in maps:
            assert hip.hipFree(p) == 0
            assert hip.hipDestroyExternalMemory(em) == 0
            os.close(fd)

    fails, retried, exported, held = 0, 0, 0, []
    log = []
    for it in range(iters):
        count = (256 * MIB) // 4 + it * 1024
        x = torch.full((count,), float(it + 1), dtype=torch.float32, device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        mine = []
        for t in (x, y):
            fd, size, attempts, base = export(t)
            fails += attempts > 0
            retried += 0 < attempts <= retry and fd >= 0
            exported += fd >= 0
            mine.append((fd, size))
            log.append([it, "x" if t is x else "y", hex(base), attempts, fd >= 0])
        # exchange: sizes and whether each fd exists, then the fds themselves
        hdr = json.dumps([[fd >= 0, size] for fd, size in mine]).encode()
        socket.send_fds(s, [hdr.ljust(256)], [fd for fd, _ in mine if fd >= 0])
        msg, fds, _, _ = socket.recv_fds(s, 256, 4)
        peer = json.loads(msg.rstrip(b" ").decode())
        for fd, _ in mine:
            if fd >= 0:
                os.close(fd)
        maps, k = [], 0
        for ok, size in peer:
            if ok:
                maps.append(imp(fds[k], size))
                k += 1
        torch.cuda.synchronize()
        s.sendall(b"1")
        s.recv(1)  # both mapped
        del x, y
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        s.sendall(b"1")
        s.recv(1)  # both freed
        if unmap == "now":
            unmap_all(maps)
        elif unmap == "late":
            unmap_all(held)
            held = maps
        else:
            held += maps
    unmap_all(held)
    q.put((rank, {"rank": rank, "iters": iters, "unmap": unmap, "retry": retry, "exports": 2 * iters,
                  "exported": exported, "failed_first_try": fails, "ok_after_retry": retried, "log": log}))


if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    unmap = sys.argv[2] if len(sys.argv) > 2 else "now"
    retry = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, iters, unmap, retry, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in sorted(res):
        print(json.dumps(res[r]))
