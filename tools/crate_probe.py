"""Where does the crate-shaped path's time go (bench.py crate_api)?

Times one RS(30,3) block of 32 MiB segments through
  wrapper      bfrs.Chunker.generate_parity (Python wrapper, bytes out)
  cabi_fresh   bfrs_generate_parity with fresh np.empty outputs (the Rust Vec shape)
  cabi_reuse   bfrs_generate_parity with reused, already-touched outputs
  objects      encoder_new / 30 x add_original_shard / encode / recovery, each timed
Prints one JSON line.  GPU box only (tools/, not a test)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "blockframe-rs_amd"))
os.environ.setdefault("BFRS_CODEC_SLOTS", "8")
import numpy as np  # noqa: E402
import bfrs  # noqa: E402
from bfrs import _ptr_array, _sz, lib  # noqa: E402

K, S, REPS = 30, 32 << 20, 5


def best(f, reps=REPS):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 2), round(float(np.median(ts)) * 1e3, 2)


def main():
    ctx = bfrs.Context(0)
    rng = np.random.default_rng(7)
    segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(K)]
    res = {"what": f"RS({K},3), {S >> 20} MiB segments, ms (best, median of {REPS})"}
    res["wrapper"] = best(lambda: bfrs.Chunker(ctx).generate_parity(segs, K, 3))
    ps, _k1 = _ptr_array([s.ctypes.data for s in segs])
    lens = (_sz * K)(*[S] * K)
    plen = _sz()

    def cabi(outs):
        po, _k2 = _ptr_array([o.ctypes.data for o in outs])
        rc = lib().bfrs_generate_parity(ctx.handle, ps, lens, K, K, 3, po, ctypes.byref(plen))
        assert rc == 0, rc

    res["cabi_fresh"] = best(lambda: cabi([np.empty(S, np.uint8) for _ in range(3)]))
    outs = [np.zeros(S, np.uint8) for _ in range(3)]
    res["cabi_reuse"] = best(lambda: cabi(outs))
    # stage by stage through the object API
    L = lib()
    stages = {"new": [], "add_all": [], "encode": [], "free": []}
    for _ in range(REPS):
        e = ctypes.c_void_p()
        t0 = time.perf_counter()
        assert L.bfrs_encoder_new(ctx.handle, K, 3, S, ctypes.byref(e)) == 0
        t1 = time.perf_counter()
        for s in segs:
            assert L.bfrs_encoder_add_original_shard(e, s.ctypes.data, S) == 0
        t2 = time.perf_counter()
        assert L.bfrs_encoder_encode(e) == 0
        t3 = time.perf_counter()
        L.bfrs_encoder_free(e)
        t4 = time.perf_counter()
        for k, v in zip(stages, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            stages[k].append(v)
    res["objects"] = {k: round(float(np.median(v)) * 1e3, 2) for k, v in stages.items()}
    gib = K * S / 2**30
    res["GiBps"] = {k: round(gib / (res[k][0] / 1e3), 2)
                    for k in ("wrapper", "cabi_fresh", "cabi_reuse")}
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
