"""How fast does this box pin host memory, and does it scale with threads?
(GPU box; measurement only.)

The archive paths pin their staging once per context: a
first commit or read spends tens of ms in hipHostMalloc.  This probe pins
N x 32 MiB buffers with hipHostMalloc from 1, 2, 4 and 8 threads (each thread
its share), and once as a single N x 32 MiB allocation, and prints GB/s of
pinned memory per variant (best of 3; buffers freed between runs)."""
import ctypes
import json
import threading
import time


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostFree.argtypes = [ctypes.c_void_p]
    hip.hipSetDevice.argtypes = [ctypes.c_int]
    assert hip.hipSetDevice(0) == 0
    S, N = 32 << 20, 16

    def pin(count, size, out):
        for _ in range(count):
            p = ctypes.c_void_p()
            assert hip.hipHostMalloc(ctypes.byref(p), size, 0) == 0
            out.append(p.value)

    def run(threads, single=False):
        bufs = []
        t0 = time.perf_counter()
        if single:
            pin(1, N * S, bufs)
        else:
            ts = [threading.Thread(target=pin, args=(N // threads, S, bufs)) for _ in range(threads)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        dt = time.perf_counter() - t0
        for p in bufs:
            assert hip.hipHostFree(ctypes.c_void_p(p)) == 0
        return N * S / dt / 1e9

    out = {}
    run(1)  # warm the runtime
    for th in (1, 2, 4, 8):
        out[f"threads_{th}"] = round(max(run(th) for _ in range(3)), 2)
    out["single_allocation"] = round(max(run(1, single=True) for _ in range(3)), 2)
    out["what"] = f"GB/s of pinned memory: {N} x {S >> 20} MiB hipHostMalloc, best of 3"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
