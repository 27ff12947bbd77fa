"""Same-process A/B of the slab wrappers' H2D shape (GPU box; measurement build).

bfrs_generate_parity / bfrs_recover_segment_rs30_3 on one RS(30,3) block of
32 MiB segments from pageable memory, as bench.py's crate_api times them,
with BFRS_SLAB_ROW_GROUP alternating between 1 (one H2D per row, round 4)
and 8 (groups of up to 8 consecutive rows as one 2-D copy), several rounds in
one process so both run on the same box, placement and host load.  Needs
BFRS_LIB=libbfrs_ab.so (the knob exists only there).  Prints one JSON line:
per variant the best and median ms of each figure over all rounds."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
os.environ.setdefault("BFRS_LIB", "libbfrs_ab.so")


def main():
    import numpy as np
    import bfrs
    assert bfrs.LIB_PATH.endswith("libbfrs_ab.so"), bfrs.LIB_PATH
    rounds = int(os.environ.get("AB_ROUNDS", "6"))
    reps = int(os.environ.get("AB_REPS", "5"))
    S, k = 32 << 20, 30
    rng = np.random.default_rng(5)
    segs = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    ctx = bfrs.Context(0)
    ch = bfrs.Chunker(ctx)
    par = [np.empty(S, np.uint8) for _ in range(3)]
    ch.generate_parity_into(segs, k, 3, par)
    target = 7
    slots = [None if i == target else segs[i] for i in range(k)]
    got = np.empty(S, np.uint8)
    variants = os.environ.get("AB_GROUPS", "1,8").split(",")
    res = {v: {"gen_touched": [], "gen_fresh": [], "rec_touched": [], "rec_fresh": []}
           for v in variants}
    ok = True

    def t(f):
        t0 = time.perf_counter()
        f()
        return (time.perf_counter() - t0) * 1e3
    t_end = time.perf_counter() + 0.5  # settle the link
    while time.perf_counter() < t_end:
        ch.generate_parity_into(segs, k, 3, par)
    for r in range(rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            os.environ["BFRS_SLAB_ROW_GROUP"] = v
            d = res[v]
            for _ in range(reps):
                d["gen_touched"].append(t(lambda: ch.generate_parity_into(segs, k, 3, par)))
                d["gen_fresh"].append(t(lambda: ch.generate_parity_into(
                    segs, k, 3, [np.empty(S, np.uint8) for _ in range(3)])))
                d["rec_touched"].append(t(lambda: bfrs.recover_segment_rs30_3_into(
                    ctx, slots, par, target, got)))
                d["rec_fresh"].append(t(lambda: bfrs.recover_segment_rs30_3_into(
                    ctx, slots, par, target, np.empty(S, np.uint8))))
            ok = ok and bool(np.array_equal(got, segs[target]))
    want = [np.empty(S, np.uint8) for _ in range(3)]
    os.environ["BFRS_SLAB_ROW_GROUP"] = "1"
    ch.generate_parity_into(segs, k, 3, want)
    ok = ok and all(np.array_equal(a, b) for a, b in zip(par, want))
    ctx.close()
    out = {v: {key: {"best": round(min(x), 2), "median": round(statistics.median(x), 2)}
               for key, x in d.items()} for v, d in res.items()}
    out["bytes_ok"] = ok
    out["what"] = (f"RS(30,3), 32 MiB pageable segments; {rounds} rounds x {reps} calls per "
                   "variant, alternating order; ms")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
