"""Config 5 of BASELINE.json: read of a corrupted large file through the
mount's read path, with GPU reconstruction and BLAKE3 (merkle leaf) re-verify,
end-to-end MB/s including host<->device copies.

The reference serves FUSE reads from src/mount/filesystem_unix.rs:176-305:
offset -> segment, cache lookup, BLAKE3 check on a miss, RS recovery of a
corrupt segment.  This drives the same core (bfrs.Archive -> libbfrs.so
bfrs_archive_read) in-process with FUSE-sized sequential reads; no kernel
FUSE mount is involved (the boxes have no libfuse), so the number excludes
the kernel round trip per read.

Steps: synthetic file -> bfrs.commit (tier 3, GPU parity) -> clean sequential
read -> corrupt `--corrupt` segments per block (bit flips, or removal with
--remove) -> fresh handle, sequential read -> check the BLAKE3 of all bytes
served against the original.  Files live under --dir (default $TMPDIR), so the
reads come from the page cache, not the device: this measures the read path,
not the disk.

Prints one JSON line.
"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-gib", type=float, default=4.0, help="SURVEY C5: 4 GiB tier-3 archive")
    ap.add_argument("--segment-bytes", type=int, default=32 << 20)
    ap.add_argument("--read-bytes", type=int, default=128 << 10, help="FUSE max_read size")
    ap.add_argument("--corrupt", type=int, default=3, help="segments damaged per block (<=3)")
    ap.add_argument("--remove", action="store_true", help="delete instead of bit-flip")
    ap.add_argument("--cache", type=int, default=64, help="segment cache capacity")
    ap.add_argument("--dir", default=None)
    args = ap.parse_args()

    ctx = bfrs.Context(0)
    work = tempfile.mkdtemp(prefix="bfrs_read_", dir=args.dir)
    try:
        n = int(args.size_gib * (1 << 30)) + 12345  # ragged tail segment
        src = os.path.join(work, "large.bin")
        rng = np.random.default_rng(5)
        with open(src, "wb") as f:
            left = n
            while left:
                c = min(left, 256 << 20)
                f.write(rng.integers(0, 256, size=c, dtype=np.uint8).tobytes())
                left -= c
        with open(src, "rb") as f:
            want = bfrs.blake3_hex(np.frombuffer(f.read(), np.uint8), threads=16)

        t0 = time.perf_counter()
        adir = bfrs.commit(ctx, src, os.path.join(work, "archive"), segment_size=args.segment_bytes)
        commit_s = time.perf_counter() - t0
        m = json.load(open(os.path.join(adir, "manifest.json")))
        assert m["original_hash"] == want

        def sweep():
            with bfrs.Archive(ctx, adir, cache_segments=args.cache) as a:
                out = np.empty(n, np.uint8)
                out[::4096] = 0  # fault the destination in before timing
                rb = args.read_bytes
                t = time.perf_counter()
                off = 0
                while off < n:  # FUSE-sized reads straight into the caller's buffer
                    off += a.read_into(off, out[off:off + rb])
                dt = time.perf_counter() - t
                return dt, a.stats(), out

        clean_s, clean_st, out = sweep()
        assert bfrs.blake3_hex(out, threads=16) == want
        del out

        rng = np.random.default_rng(6)
        damaged = 0
        for b, blk in m["merkle_tree"]["blocks"].items():
            k = len(blk["segments"])
            for s in rng.choice(k, size=min(args.corrupt, k), replace=False):
                p = os.path.join(adir, "blocks", f"block_{b}", "segments", f"segment_{s}.dat")
                if args.remove:
                    os.remove(p)
                else:
                    with open(p, "r+b") as f:
                        f.seek(int(rng.integers(0, os.path.getsize(p))))
                        c = f.read(1)
                        f.seek(-1, 1)
                        f.write(bytes([c[0] ^ 0xFF]))
                damaged += 1

        dirty_s, dirty_st, out = sweep()
        ok = bfrs.blake3_hex(out, threads=16) == want
        print(json.dumps({
            "metric": "end-to-end read MB/s of a corrupted large file (config 5)",
            "value": round(n / dirty_s / 1e6, 1), "unit": "MB/s",
            "clean_read_MBps": round(n / clean_s / 1e6, 1),
            "commit_MBps": round(n / commit_s / 1e6, 1),
            "bytes": n, "segment_bytes": args.segment_bytes, "read_bytes": args.read_bytes,
            "blocks": len(m["merkle_tree"]["blocks"]), "damaged_segments": damaged,
            "damage": "removed" if args.remove else "bit-flip",
            "stats_dirty": dirty_st, "stats_clean": clean_st, "blake3_match": ok,
            "source": "page cache (files written by this run)",
        }))
        if not ok:
            sys.exit(1)
    finally:
        shutil.rmtree(work, ignore_errors=True)
        ctx.close()


if __name__ == "__main__":
    main()
