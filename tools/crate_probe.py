"""Where does the crate-shaped path's time go (bench.py crate_api)?

Times one RS(30,3) block of 32 MiB segments, best / median of REPS, in ms:
  cabi_fresh_<mode>   bfrs_generate_parity into fresh np.empty outputs (the
                      Rust Vec shape), BFRS_CODEC_STAGING=<mode>
  cabi_reuse_<mode>   the same into reused, already-touched outputs
  recover_fresh/reuse bfrs_recover_segment_rs30_3 likewise (direct staging)
  objects             encoder_new / 30 x add_original_shard / encode / free
  touch_96MiB         first touch of 3 fresh 32 MiB numpy buffers (1 thread)
  d2h_fresh/touched   torch D2H of 96 MiB into a fresh / touched pageable buffer
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


def best(f, reps=REPS, prep=None):
    ts = []
    for _ in range(reps):
        arg = prep() if prep else None
        t0 = time.perf_counter()
        f(arg) if prep else f()
        ts.append(time.perf_counter() - t0)
    return round(min(ts) * 1e3, 2), round(float(np.median(ts)) * 1e3, 2)


def context(mode):
    old = os.environ.get("BFRS_CODEC_STAGING")
    os.environ["BFRS_CODEC_STAGING"] = mode
    try:
        return bfrs.Context(0)
    finally:
        if old is None:
            del os.environ["BFRS_CODEC_STAGING"]
        else:
            os.environ["BFRS_CODEC_STAGING"] = old


def main():
    import torch
    if len(sys.argv) > 1:  # GiB of torch pinned host memory allocated (and freed) first, as bench.py's pcie_inclusive does
        gib = float(sys.argv[1])
        t = torch.empty(int(gib * 2**30), dtype=torch.uint8, pin_memory=True)
        t.fill_(1)
        del t
    rng = np.random.default_rng(7)
    segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(K)]
    if os.environ.get("PROBE_TORCH_SEGS"):  # segments as bench.py makes them: .cpu() of device rows
        dev = torch.from_numpy(np.stack(segs)).cuda()
        segs = [dev[i].cpu().numpy() for i in range(K)]
        del dev
    res = {"what": f"RS({K},3), {S >> 20} MiB segments, ms (best, median of {REPS})"}
    ps, _k1 = _ptr_array([s.ctypes.data for s in segs])
    lens = (_sz * K)(*[S] * K)
    plen = _sz()
    for mode in ("direct", "pinned"):
        ctx = context(mode)

        def cabi(outs):
            po, _k2 = _ptr_array([o.ctypes.data for o in outs])
            rc = lib().bfrs_generate_parity(ctx.handle, ps, lens, K, K, 3, po, ctypes.byref(plen))
            assert rc == 0, rc

        res[f"cabi_fresh_{mode}"] = best(lambda: cabi([np.empty(S, np.uint8) for _ in range(3)]))

        # fresh INPUT buffers too (untimed copies): BlockFrame's segments are
        # new mmap'd file pages for every block, never seen by HIP before
        def fresh_inputs():
            return [np.array(x) for x in segs]

        def cabi_new_inputs(xs):
            p2, _k3 = _ptr_array([x.ctypes.data for x in xs])
            outs_now = outs_fresh()  # kept alive across the call
            po, _k2 = _ptr_array([o.ctypes.data for o in outs_now])
            rc = lib().bfrs_generate_parity(ctx.handle, p2, lens, K, K, 3, po, ctypes.byref(plen))
            assert rc == 0, rc

        def outs_fresh():
            return [np.empty(S, np.uint8) for _ in range(3)]
        res[f"cabi_fresh_inputs_{mode}"] = best(cabi_new_inputs, prep=fresh_inputs)
        outs = [np.zeros(S, np.uint8) for _ in range(3)]
        res[f"cabi_reuse_{mode}"] = best(lambda: cabi(outs))
        if mode == "direct":
            par = outs
            slots = [None if i == 4 else segs[i] for i in range(K)]
            res["recover_fresh"] = best(lambda: bfrs.recover_segment_rs30_3_into(
                ctx, slots, par, 4, np.empty(S, np.uint8)))
            out = np.zeros(S, np.uint8)
            res["recover_reuse"] = best(lambda: bfrs.recover_segment_rs30_3_into(
                ctx, slots, par, 4, out))
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
        ctx.close()

    def touch():
        for _ in range(3):
            a = np.empty(S, np.uint8)
            a[::4096] = 0
    res["touch_96MiB"] = best(touch)
    dev = torch.empty(3 * S, dtype=torch.uint8, device="cuda")

    def d2h(fresh):
        h = torch.from_numpy(np.empty(3 * S, np.uint8) if fresh else keep)
        torch.cuda.synchronize()
        h.copy_(dev)
    keep = np.ones(3 * S, np.uint8)
    res["d2h_fresh"] = best(lambda: d2h(True))
    res["d2h_touched"] = best(lambda: d2h(False))
    gib = K * S / 2**30
    res["GiBps"] = {k: round(gib / (v[0] / 1e3), 2) for k, v in res.items()
                    if k.startswith("cabi_")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
