"""How fast does this box pin host memory, and does it scale with threads?
(GPU box; measurement only.)

The archive paths pin their staging once per context: a
first commit or read spends tens of ms in hipHostMalloc.  This probe pins
N x 32 MiB buffers with hipHostMalloc from 1, 2, 4 and 8 threads (each thread
its share), and once as a single N x 32 MiB allocation, and prints GB/s of
pinned memory per variant (best of 3; buffers freed between runs).

Round 6 adds the registration forms (the fresh-context
read pins its segment pool at ~5-6 GB/s): anonymous mmap + first touch +
hipHostRegister, with and without MADV_HUGEPAGE (2 MiB pages: 512x fewer
pages to lock and map for the GPU), and hipHostMalloc with the non-coherent
and NUMA-user flags; the first-touch share of each is timed apart."""
import ctypes
import json
import mmap
import threading
import time

MADV_HUGEPAGE = 14


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    libc.memset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipSetDevice.argtypes = [ctypes.c_int]
    assert hip.hipSetDevice(0) == 0
    S, N = 32 << 20, 16

    def pin(count, size, out, flags=0):
        for _ in range(count):
            p = ctypes.c_void_p()
            assert hip.hipHostMalloc(ctypes.byref(p), size, flags) == 0
            out.append(p.value)

    def run(threads, single=False, flags=0):
        bufs = []
        t0 = time.perf_counter()
        if single:
            pin(1, N * S, bufs, flags)
        else:
            ts = [threading.Thread(target=pin, args=(N // threads, S, bufs, flags))
                  for _ in range(threads)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        dt = time.perf_counter() - t0
        for p in bufs:
            assert hip.hipHostFree(ctypes.c_void_p(p)) == 0
        return N * S / dt / 1e9

    def register(huge, per_buffer=True):
        """mmap (+ MADV_HUGEPAGE) + touch + hipHostRegister; returns
        (GB/s overall, GB/s of the register step alone)."""
        size = S if per_buffer else N * S
        count = N if per_buffer else 1
        t0 = time.perf_counter()
        maps, t_reg = [], 0.0
        for _ in range(count):
            p = libc.mmap(None, size, mmap.PROT_READ | mmap.PROT_WRITE,
                          mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS, -1, 0)
            assert p not in (None, ctypes.c_void_p(-1).value)
            if huge:
                libc.madvise(p, size, MADV_HUGEPAGE)
            libc.memset(p, 0, size)  # first touch
            t1 = time.perf_counter()
            assert hip.hipHostRegister(ctypes.c_void_p(p), size, 0) == 0
            t_reg += time.perf_counter() - t1
            maps.append(p)
        dt = time.perf_counter() - t0
        for p in maps:
            assert hip.hipHostUnregister(ctypes.c_void_p(p)) == 0
            libc.munmap(p, size)
        return N * S / dt / 1e9, N * S / t_reg / 1e9

    out = {}
    run(1)  # warm the runtime
    for th in (1, 2, 4, 8):
        out[f"threads_{th}"] = round(max(run(th) for _ in range(3)), 2)
    out["single_allocation"] = round(max(run(1, single=True) for _ in range(3)), 2)
    for name, fl in (("noncoherent", 0x80000000), ("numa_user", 0x20000000)):
        try:
            out[f"hipHostMalloc_{name}"] = round(max(run(1, flags=fl) for _ in range(3)), 2)
        except AssertionError:
            out[f"hipHostMalloc_{name}"] = "failed"
    for huge in (False, True):
        for per in (True, False):
            r = [register(huge, per) for _ in range(3)]
            best = max(r)
            out[f"register_{'huge' if huge else '4k'}_{'per32MiB' if per else 'single'}"] = {
                "GBps": round(best[0], 2), "register_only_GBps": round(best[1], 2)}
    out["what"] = (f"GB/s of pinned memory: {N} x {S >> 20} MiB, best of 3; register_*: anonymous "
                   "mmap (+ MADV_HUGEPAGE) + memset + hipHostRegister, the register step alone beside it")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
