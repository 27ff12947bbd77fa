"""Throughput of the archive pipeline per tier: bfrs_commit of a tier-1
(24 MB), tier-2 (1 GB) and tier-3 (4 GiB) file, then bfrs_repair of the
tier-3 archive with 3 damaged segments per block, and bfrs_health_check.
Files live under --dir (default $TMPDIR, page cache).  One JSON line."""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
import bfrs  # noqa: E402


def make(path, n, seed):
    rng = np.random.default_rng(seed)
    with open(path, "wb") as f:
        left = n
        while left:
            c = min(left, 256 << 20)
            f.write(rng.integers(0, 256, size=c, dtype=np.uint8).tobytes())
            left -= c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=None)
    ap.add_argument("--t3-gib", type=float, default=4.0)
    a = ap.parse_args()
    ctx = bfrs.Context(0)
    work = tempfile.mkdtemp(prefix="bfrs_commit_", dir=a.dir)
    res = {}
    try:
        for tier, n in [(1, 24_000_000), (2, 1_000_000_000), (3, int(a.t3_gib * (1 << 30)))]:
            src = os.path.join(work, f"t{tier}.bin")
            make(src, n, tier)
            t = time.perf_counter()
            adir = bfrs.commit(ctx, src, os.path.join(work, "archive"))
            dt = time.perf_counter() - t
            m = json.load(open(os.path.join(adir, "manifest.json")))
            assert m["tier"] == tier
            res[f"commit_tier{tier}_MBps"] = round(n / dt / 1e6, 1)
            # again, into another root: the context's staging is in place now
            t = time.perf_counter()
            again = bfrs.commit(ctx, src, os.path.join(work, "again"))
            res[f"commit_tier{tier}_again_MBps"] = round(n / (time.perf_counter() - t) / 1e6, 1)
            m2 = json.load(open(os.path.join(again, "manifest.json")))
            assert m2["merkle_tree"] == m["merkle_tree"] and m2["original_hash"] == m["original_hash"]
            shutil.rmtree(os.path.join(work, "again"))
            os.remove(src)
            if tier == 2:  # every data and parity file hashed (tiers 1/2: on the host threads)
                t = time.perf_counter()
                assert bfrs.health_check(ctx, adir)["status"] == "Healthy"
                res["health_check_tier2_MBps"] = round(n / (time.perf_counter() - t) / 1e6, 1)
                t = time.perf_counter()  # nothing to restore: every file verified
                assert bfrs.repair(ctx, adir)["segments_repaired"] == 0
                res["repair_tier2_clean_MBps"] = round(n / (time.perf_counter() - t) / 1e6, 1)
            if tier == 3:
                rng = np.random.default_rng(7)
                damaged = 0
                for b, blk in m["merkle_tree"]["blocks"].items():
                    for s in rng.choice(len(blk["segments"]), size=3, replace=False):
                        p = os.path.join(adir, "blocks", f"block_{b}", "segments", f"segment_{s}.dat")
                        with open(p, "r+b") as f:
                            f.seek(100)
                            c = f.read(1)
                            f.seek(100)
                            f.write(bytes([c[0] ^ 1]))
                        damaged += 1
                t = time.perf_counter()
                h = bfrs.health_check(ctx, adir)
                res["health_check_tier3_MBps"] = round(n / (time.perf_counter() - t) / 1e6, 1)
                assert h["status"] == "Recoverable", h["status"]
                t = time.perf_counter()
                rep = bfrs.repair(ctx, adir)
                res["repair_tier3_MBps"] = round(n / (time.perf_counter() - t) / 1e6, 1)
                assert rep["segments_repaired"] == damaged, rep
                assert bfrs.health_check(ctx, adir)["status"] == "Healthy"
                res["repair_damaged_segments"] = damaged
        print(json.dumps({"metric": "archive pipeline MB/s (file bytes / wall time)", **res,
                          "source": "page cache (files written by this run)"}))
    finally:
        shutil.rmtree(work, ignore_errors=True)
        ctx.close()


if __name__ == "__main__":
    main()
