"""GPU soak of the archive pipeline (commit / health check / read / repair),
a test tool in the spirit of tools/soak.py.

Each case commits a random file (tier 1, 2 or 3 forced; segment sizes of
64 / 96 / 128 KiB, so tier-3 last blocks of every size 1..30 come up; file
sizes on and around segment boundaries), damages random shards (flip a byte,
delete, truncate), and checks against a model of what must happen:
  - recoverable (tier 3: damaged data <= valid parity in every block; tiers
    1/2: data or one parity copy valid per segment): the health check says
    recoverable, a sequential read in random-sized requests returns the
    original bytes, repair reports no unrecoverable block, the archive is
    Healthy afterwards and reads back the original again;
  - unrecoverable: the health check says so and repair counts it;
  - a tier-3 file whose last block is ONE odd-length segment: commit fails
    with BFRS_E_INVALID_SHARD_SIZE and leaves no *_computing directory
    (generate.rs:84, commit.rs:440-441).
Prints one JSON line; exit 1 on any violation.

usage: python3 tools/soak_archive.py [--seconds 90] [--readers 4] [--workdir /tmp]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=90.0)
    ap.add_argument("--seed", type=int, default=0xA4C1)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--readers", type=int, default=4, help="threads sharing one read handle")
    a = ap.parse_args()
    import numpy as np
    import bfrs

    ctx = bfrs.Context(0)
    rng = np.random.default_rng(a.seed)
    stats = {"cases": 0, "by_tier": {}, "recoverable": 0, "unrecoverable": 0, "odd_last_block": 0,
             "bytes_committed": 0, "failures": []}
    stop = time.perf_counter() + a.seconds

    def fail(case, what):
        if len(stats["failures"]) < 20:
            stats["failures"].append({**case, "what": what})

    def damage(path):
        """Damage one shard file: flip a byte, delete it, or truncate it."""
        act = str(rng.choice(["flip", "delete", "truncate"]))
        if not os.path.exists(path):
            return
        if act == "delete":
            os.remove(path)
        elif act == "truncate":
            n = os.path.getsize(path)
            with open(path, "r+b") as f:
                f.truncate(n // 2)
        else:
            with open(path, "r+b") as f:
                n = os.path.getsize(path)
                at = int(rng.integers(0, max(1, n)))
                f.seek(at)
                c = f.read(1)
                f.seek(at)
                f.write(bytes([(c[0] if c else 0) ^ 0x5A]))

    def read_all(adir, n):
        out = np.empty(n, np.uint8)
        with bfrs.Archive(ctx, adir, cache_segments=8) as ar:
            off = 0
            while off < n:
                want = int(rng.integers(1, 3 * 128 * 1024))
                got = ar.read_into(off, out[off:off + want])
                if got <= 0:
                    raise RuntimeError(f"short read at {off}")
                off += got
        return out

    while time.perf_counter() < stop:
        tier = int(rng.choice([1, 2, 3, 3, 3]))
        S = int(rng.choice([64 << 10, 96 << 10, 128 << 10]))
        if tier == 1:
            n = int(rng.integers(1, 3 * S))
        elif tier == 2:
            nseg = int(rng.integers(1, 11))
            n = (nseg - 1) * S + int(rng.choice([1, 2, 63, 64, S - 1, S, int(rng.integers(1, S + 1))]))
        else:
            nseg = int(rng.choice([1, 2, 3, 4, 29, 30, 31, 34, 60, 61, int(rng.integers(1, 76))]))
            n = (nseg - 1) * S + int(rng.choice([1, 2, 63, 64, S - 1, S, int(rng.integers(1, S + 1))]))
        case = {"tier": tier, "S": S, "n": n}
        work = tempfile.mkdtemp(prefix="bfrs_soak_", dir=a.workdir)
        try:
            data = rng.integers(0, 256, n, dtype=np.uint8)
            src = os.path.join(work, "f.bin")
            data.tofile(src)
            root = os.path.join(work, "store")
            nseg = -(-n // S)
            odd_last = tier == 3 and nseg % 30 == 1 and (n - (nseg - 1) * S) % 2 == 1
            try:
                adir = bfrs.commit(ctx, src, root, segment_size=S, tier=tier)
            except bfrs.BfrsError as e:
                if odd_last and e.code == bfrs.E_INVALID_SHARD_SIZE and \
                        not any(x.endswith("_computing") for x in os.listdir(root)):
                    stats["odd_last_block"] += 1
                else:
                    fail(case, f"commit: {e.code} {e}")
                continue
            if odd_last:
                fail(case, "commit accepted an odd single-segment last block")
                continue
            stats["bytes_committed"] += n
            if bfrs.health_check(ctx, adir)["status"] != "Healthy":
                fail(case, "fresh archive not Healthy")
                continue
            # damage, and the model of recoverability
            recoverable = True
            if tier == 3:
                nblocks = -(-nseg // 30)
                for b in sorted(rng.choice(nblocks, int(rng.integers(1, min(3, nblocks) + 1)),
                                           replace=False).tolist()):
                    k = min(30, nseg - 30 * b)
                    nd = int(rng.integers(0, min(4, k) + 1))
                    npar = int(rng.integers(0, 4 - min(nd, 3) + (1 if rng.random() < 0.15 else 0)))
                    npar = min(npar, 3)
                    for s in rng.choice(k, nd, replace=False).tolist():
                        damage(os.path.join(adir, "blocks", f"block_{b}", "segments", f"segment_{s}.dat"))
                    for p in rng.choice(3, npar, replace=False).tolist():
                        damage(os.path.join(adir, "blocks", f"block_{b}", "parity", f"block_parity_{p}.dat"))
                    recoverable &= nd <= 3 - npar
            else:
                units = 1 if tier == 1 else nseg
                for u in sorted(rng.choice(units, int(rng.integers(1, min(3, units) + 1)),
                                           replace=False).tolist()):
                    dmg_data = rng.random() < 0.8
                    npar = int(rng.integers(0, 3 + (1 if rng.random() < 0.15 else 0)))
                    if tier == 1:
                        dpath = os.path.join(adir, "data.dat")
                        ppath = [os.path.join(adir, f"parity_{p}.dat") for p in range(3)]
                    else:
                        dpath = os.path.join(adir, "segments", f"segment_{u}.dat")
                        ppath = [os.path.join(adir, "parity", f"segment_{u}_parity_{p}.dat") for p in range(3)]
                    if dmg_data:
                        damage(dpath)
                    for p in rng.choice(3, npar, replace=False).tolist():
                        damage(ppath[p])
                    recoverable &= (not dmg_data) or npar < 3
            h = bfrs.health_check(ctx, adir)
            if bool(h["recoverable"]) != recoverable:
                fail(case, f"health_check recoverable={h['recoverable']} model={recoverable} ({h['status']})")
                continue
            if recoverable:
                stats["recoverable"] += 1
                if a.readers > 1 and rng.random() < 0.5:
                    # several threads reading random ranges through ONE handle
                    # (prefetch and reconstruction shared between them)
                    errs = []
                    with bfrs.Archive(ctx, adir, cache_segments=4) as ar:
                        def reader(seed):
                            r = np.random.default_rng(seed)
                            for _ in range(16):
                                off = int(r.integers(0, n))
                                ln = int(r.integers(1, min(n - off, 3 * S) + 1))
                                got = ar.read(off, ln)
                                if got != data[off:off + ln].tobytes():
                                    errs.append((off, ln))
                        th = [threading.Thread(target=reader, args=(int(rng.integers(1 << 30)),))
                              for _ in range(a.readers)]
                        for t in th:
                            t.start()
                        for t in th:
                            t.join()
                    stats["concurrent_reads"] = stats.get("concurrent_reads", 0) + 1
                    if errs:
                        fail(case, f"concurrent reads differ at {errs[:3]}")
                        continue
                if not np.array_equal(read_all(adir, n), data):
                    fail(case, "read of the damaged archive differs")
                    continue
                rep = bfrs.repair(ctx, adir)
                if rep["unrecoverable_blocks"]:
                    fail(case, f"repair: {rep}")
                    continue
                if bfrs.health_check(ctx, adir)["status"] != "Healthy":
                    fail(case, "not Healthy after repair")
                    continue
                if not np.array_equal(read_all(adir, n), data):
                    fail(case, "read after repair differs")
                    continue
            else:
                stats["unrecoverable"] += 1
                rep = bfrs.repair(ctx, adir)
                if not rep["unrecoverable_blocks"]:
                    fail(case, f"repair did not count the unrecoverable unit: {rep}")
        except Exception as e:  # noqa: BLE001 -- any other error is a violation
            fail(case, f"{type(e).__name__}: {e}")
        finally:
            if stats["cases"] % 200 == 0:  # progress on stderr (long runs must keep writing)
                print(f"progress: {stats['cases']} cases, {len(stats['failures'])} failures",
                      file=sys.stderr, flush=True)
            stats["cases"] += 1
            stats["by_tier"][str(tier)] = stats["by_tier"].get(str(tier), 0) + 1
            shutil.rmtree(work, ignore_errors=True)
    ctx.close()
    stats["seconds"] = a.seconds
    print(json.dumps(stats))
    return 1 if stats["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
