"""Generates tests/golden/*.json from the oracle (oracle/rs_oracle.c).

The reference pins no parity bytes and its crate cannot be
built here, so golden vectors come from the oracle restatement, which is
itself pinned to SURVEY Appendix A.7's independently computed KAT (checked in
tests/test_oracle.py before these fixtures are trusted).

  python tests/golden/make_golden.py            # small vectors (seconds)
  python tests/golden/make_golden.py --large    # config-size digests (minutes)
  python tests/golden/make_golden.py --r2       # RS(3,3)/RS(4,3) under both rates
  python tests/golden/make_golden.py --blake3   # BLAKE3 of C2's 128 segments (bench.py)
"""
import argparse
import hashlib
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))

import oracle as O  # noqa: E402
from bfrs import synth  # noqa: E402

# (k, m, shard_bytes) small cases: BlockFrame shapes, LowRate shapes, tails.
SMALL_CASES = [
    (30, 3, 128), (30, 3, 64), (8, 3, 64), (20, 3, 192), (1, 3, 64), (2, 3, 128),
    (3, 3, 64), (4, 3, 64), (5, 3, 64), (29, 3, 64), (30, 3, 70), (7, 3, 2), (30, 3, 1000),
    (1, 3, 8000002 % 4096 + 2), (16, 4, 128), (10, 1, 64), (64, 3, 64), (65, 5, 128),
    # LowRate with zero-padded originals (k not a power of two): round 2
    (3, 5, 64), (7, 5, 128), (5, 9, 64),
]


def small():
    rng = np.random.default_rng(0xB10C)
    cases = []
    for k, m, n in SMALL_CASES:
        orig = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
        rec = O.encode(orig, m)
        entry = {"k": k, "m": m, "shard_bytes": n,
                 "originals": [o.tobytes().hex() for o in orig],
                 "recovery": [r.tobytes().hex() for r in rec],
                 "decodes": []}
        # a few erasure patterns, plus one with an inconsistent (corrupted)
        # recovery shard: pins the crate decoder's exact linear map.
        pats = []
        e = min(m, k)
        for er in itertools.islice(itertools.combinations(range(k + m), e), 0, 3):
            pats.append(list(er))
        pats.append(sorted(rng.choice(k, size=min(e, k), replace=False).tolist()))
        for pi, er in enumerate(pats):
            o = [None if i in er else orig[i] for i in range(k)]
            r = [None if (k + j) in er else rec[j] for j in range(m)]
            if all(x is not None for x in o):
                continue
            corrupt = pi == len(pats) - 1 and any(x is not None for x in r)
            if corrupt:
                j = next(j for j in range(m) if r[j] is not None)
                bad = r[j].copy()
                bad[::7] ^= 0x5A
                r = list(r)
                r[j] = bad
            out = O.decode(o, r)
            entry["decodes"].append({
                "erased": er, "corrupt_recovery": corrupt,
                "recovery_used": [None if x is None else x.tobytes().hex() for x in r],
                "restored": {str(i): a.tobytes().hex() for i, a in out.items()},
            })
        cases.append(entry)
    with open(os.path.join(HERE, "rs_small.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "rng": "numpy PCG64 seed 0xB10C",
                   "cases": cases}, f)


def large(threads):
    """C2 (128 x 32 MiB, 4xRS(30,3)+RS(8,3)) and C4 (320 segments) parity digests."""
    out = {}
    for name, nseg, seed in (("c2_128x32MiB", 128, 0xB10C), ("c4_320x32MiB", 320, 0xB10C)):
        shapes = synth.block_shapes(nseg)
        digests = []
        seg = 0
        for b, k in enumerate(shapes):
            data = [synth.segment_np(seed, seg + i, synth.SEGMENT_SIZE) for i in range(k)]
            seg += k
            rec = O.encode(data, 3, engine=O.ENGINE_AVX2 if O.lib().oracle_have_avx2() else 0)
            digests.append([hashlib.sha256(r.tobytes()).hexdigest() for r in rec])
            print(name, b, k, digests[-1][0][:16], flush=True)
        out[name] = {"seed": seed, "segments": nseg, "segment_size": synth.SEGMENT_SIZE,
                     "blocks": shapes, "parity_sha256": digests}
    with open(os.path.join(HERE, "rs_large.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --large",
                   "synth": "blockframe-rs_amd/bfrs/synth.py splitmix64", **out}, f, indent=1)


def blake3_c2():
    """BLAKE3 of each of C2's 128 data segments (seed 0xB10C), by the oracle's
    BLAKE3 (pinned to the reference KAT, src/utils.rs:17-18): the golden of
    bench.py's device-BLAKE3 sub-object (the per-segment hashes a tier-3
    commit writes into the manifest, commit.rs:429)."""
    digests = []
    for i in range(128):
        digests.append(O.blake3_hex(synth.segment_np(0xB10C, i, synth.SEGMENT_SIZE)))
    with open(os.path.join(HERE, "blake3_c2.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --blake3",
                   "synth": "blockframe-rs_amd/bfrs/synth.py splitmix64", "seed": 0xB10C,
                   "segments": 128, "segment_size": synth.SEGMENT_SIZE,
                   "blake3": digests}, f, indent=1)


def r2():
    """Risk r2: which rate DefaultRate picks for k in {3, 4}
    at m = 3 decides the parity bytes of a tier-3 file whose last block holds
    3 or 4 segments.  No reference-held vector settles it, so these fixtures
    carry BOTH rates' parity and decodes, labelled, plus the rate this build
    chose (plan.cpp choose_rate): a run of the real crate on the same inputs
    settles the question by matching exactly one of them."""
    rng = np.random.default_rng(0x52)
    cases = []
    for k in (3, 4):
        for n in (128, 70):
            orig = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
            # the bench's 3-erasure pattern: originals 0..2 missing
            er = list(range(min(3, k)))
            per = {}
            for name, rate in (("low", O.RATE_LOW), ("high", O.RATE_HIGH)):
                rec = O.encode(orig, 3, rate=rate)
                o = [None if i in er else orig[i] for i in range(k)]
                out = O.decode(o, rec, rate=rate)
                assert all(np.array_equal(out[i], orig[i]) for i in er)
                per[name] = {"recovery": [r.tobytes().hex() for r in rec]}
            cases.append({
                "k": k, "m": 3, "shard_bytes": n,
                "originals": [x.tobytes().hex() for x in orig],
                "erased": er,
                "rates": per,
                "this_build_default": "high" if O.use_high_rate(k, 3) else "low",
            })
    with open(os.path.join(HERE, "rs_r2.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --r2",
                   "rng": "numpy PCG64 seed 0x52",
                   "label": "r2-dependent: parity of RS(3,3) and RS(4,3) under LowRate and HighRate; "
                            "which one the reed-solomon-simd 3.1.0 DefaultRate produces is unpinned "
                            "here (no crate, no reference vector)",
                   "cases": cases}, f, indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true")
    ap.add_argument("--r2", action="store_true")
    ap.add_argument("--blake3", action="store_true")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    if a.large:
        large(a.threads)
    elif a.r2:
        r2()
    elif a.blake3:
        blake3_c2()
    else:
        small()
