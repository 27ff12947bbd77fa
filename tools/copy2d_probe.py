"""H2D copy shapes for a slab of a strided shard set (GPU box; measurement only).

A host batch moves, per 8 MiB column slab, one piece of each of k shard rows
to HBM (runtime.cpp run_host).  When the rows sit at a constant pitch (a
pinned tensor, or BlockFrame's mmap'd file: segments S apart), the k pieces
are one 2-D copy.  This probe times, for k = 30 rows of 32 MiB in pinned
memory, over 3 streams like the pipeline:
  rows    k hipMemcpyAsync of the slab width per slab (what run_host does)
  two_d   one hipMemcpy2DAsync per slab (height k)
  whole   k whole-row copies (one 32 MiB copy per row, no slabs)
and each again with the parity D2H of the previous slab on the same stream
(3 rows per slab back to pinned memory), the pipeline's duplex shape.
Prints one JSON line of GB/s (H2D bytes / time, best of 5)."""
import ctypes
import json
import time

import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_void_p]
    hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                     ctypes.c_int, ctypes.c_void_p]
    H2D, D2H = 1, 2
    k, S, slab, m = 30, 32 << 20, 8 << 20, 3
    host = torch.empty(k, S, dtype=torch.uint8, pin_memory=True)
    host.copy_(torch.randint(0, 256, (k, S), dtype=torch.uint8))
    hpar = torch.empty(m, S, dtype=torch.uint8, pin_memory=True)
    dev = [torch.empty(k + m, slab, dtype=torch.uint8, device="cuda") for _ in range(3)]
    dwhole = torch.empty(k, S, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(3)]

    def run(shape, duplex):
        for q in range(S // slab):
            st = streams[q % 3]
            h = st.cuda_stream
            d = dev[q % 3]
            off = q * slab
            if shape == "rows":
                for i in range(k):
                    rc = hip.hipMemcpyAsync(d[i].data_ptr(), host[i].data_ptr() + off, slab, H2D, h)
                    assert rc == 0, rc
            else:
                rc = hip.hipMemcpy2DAsync(d.data_ptr(), slab, host.data_ptr() + off, S, slab, k,
                                          H2D, h)
                assert rc == 0, rc
            if duplex:
                for j in range(m):
                    rc = hip.hipMemcpyAsync(hpar[j].data_ptr() + off, d[k + j].data_ptr(), slab,
                                            D2H, h)
                    assert rc == 0, rc

    def run_whole(duplex):
        h = streams[0].cuda_stream
        for i in range(k):
            assert hip.hipMemcpyAsync(dwhole[i].data_ptr(), host[i].data_ptr(), S, H2D, h) == 0
        if duplex:
            h2 = streams[1].cuda_stream
            for j in range(m):
                assert hip.hipMemcpyAsync(hpar[j].data_ptr(), dwhole[j].data_ptr(), S, D2H, h2) == 0

    def best(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return round(k * S / min(ts) / 1e9, 2)

    out = {}
    for duplex in (False, True):
        tag = "_duplex" if duplex else ""
        out["rows" + tag] = best(lambda: run("rows", duplex))
        out["two_d" + tag] = best(lambda: run("two_d", duplex))
        out["whole" + tag] = best(lambda: run_whole(duplex))
    # the 2-D copy must move the same bytes
    run("two_d", False)
    torch.cuda.synchronize()
    out["two_d_bytes_ok"] = bool(torch.equal(dev[(S // slab - 1) % 3][:k].cpu(),
                                             host[:, S - slab:]))
    out["what"] = (f"H2D GB/s of {k} pinned rows of {S >> 20} MiB in {slab >> 20} MiB slabs "
                   "over 3 streams (best of 5); _duplex: + 3 rows of D2H per slab")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
