"""GPU soak test (measurement/test tool; the oracle is the checker only).

For a fixed wall time, T threads share ONE context whose plan cache is capped
small (BFRS_PLAN_CACHE, default 16) so plans are evicted while other threads'
batches hold theirs.  Every case draws a random shape (k <= 64, m <= 8,
shard bytes even incl. tails, 0..m erasures, sometimes a corrupted recovery
shard) and one entry point (one-shot host API, host batch of 1-4 blocks,
device batch of 1-4 blocks, the encoder/decoder objects), runs it on the GPU and compares every output
byte with oracle/rs_oracle.c.  Prints one JSON line; exit 1 on any mismatch.

usage: BFRS_PLAN_CACHE=16 python3 tools/soak.py [--seconds 60] [--threads 4]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0x50A4)
    ap.add_argument("--large", action="store_true", help="10%% of cases with 1-3 MiB shards")
    ap.add_argument("--huge", type=float, default=0.0,
                    help="this fraction of cases with 8-40 MiB shards (k <= 6, ragged sizes): "
                         "the threaded staging copies and their shared budget (host_copy.cpp)")
    ap.add_argument("--maps", default=None,
                    help="write /proc/self/maps here after the context opens and again at the "
                         "end, so the raw PCs of a fault handler's stack resolve to DSO + offset "
                         "(default: gpurun_out/soak_<pid>.maps if gpurun_out/ exists)")
    a = ap.parse_args()
    if a.maps is None and os.path.isdir("gpurun_out"):
        a.maps = f"gpurun_out/soak_{os.getpid()}.maps"

    def write_maps(tag):
        if a.maps:
            with open("/proc/self/maps") as f, open(a.maps, "w") as o:
                o.write(f"# {tag}, pid {os.getpid()}\n" + f.read())
    os.environ.setdefault("BFRS_PLAN_CACHE", "16")
    import numpy as np
    import torch
    import bfrs
    import oracle

    ctx = bfrs.Context(0)
    write_maps("after bfrs_open")
    stats = {"cases": 0, "bytes": 0, "by_api": {}, "failures": []}
    lock = threading.Lock()
    # What every thread is running right now (case number, API, shape, start
    # time): snapshotted at the first failure, so a sticky, asynchronously
    # reported HIP error is recorded with everything that was in flight on
    # the context when it surfaced (DESIGN.md §7c, round 4's fault)
    inflight = {}
    t_zero = time.perf_counter()
    stop = time.perf_counter() + a.seconds

    def one_block(rng):
        k = int(rng.choice([1, 2, 3, 4, 5, 8, 20, 30, int(rng.integers(1, 65))]))
        m = int(rng.choice([1, 2, 3, 3, 3, 4, int(rng.integers(1, 9))]))
        return k, m

    def worker(tid):
        rng = np.random.default_rng(a.seed + tid)
        stream = torch.cuda.Stream()
        while time.perf_counter() < stop:
            api = str(rng.choice(["host", "host_batch", "dev_batch", "objects", "wrappers"]))
            k, m = one_block(rng)
            huge = a.huge > 0 and rng.random() < a.huge
            if api == "wrappers" and rng.random() < 0.5 and not huge:  # recover_segment_rs30_3's shape
                k, m = 30, 3
            nblocks = 1 if api in ("host", "objects", "wrappers") else int(rng.integers(1, 5))
            n = int(rng.choice([64, 128, 4096, 65536, int(rng.integers(1, 3000)) * 2]))
            if a.large and rng.random() < 0.1:  # multi-tile grids: 1-3 MiB with a ragged tail
                n = int(rng.integers(1, 4)) * (1 << 20) + int(rng.integers(0, 64)) * 2
            if huge:  # 8-40 MiB, any even size: staging copies split into parts with remainders
                k, m, nblocks = min(k, 6), min(m, 3), 1
                n = int(rng.integers(4 << 20, 20 << 20)) * 2
                if api == "wrappers" and rng.random() < 0.3:  # the slab-pipelined recover too
                    k, m, n = 30, 3, int(rng.integers(8 << 20, 10 << 20)) * 2
            blocks = []
            for _ in range(nblocks):
                data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
                rec = oracle.encode(data, m, oracle.ENGINE_AVX2)
                ne = int(rng.integers(0, m + 1))
                er = sorted(rng.choice(k, min(ne, k), replace=False).tolist()) if ne else []
                # keep k shards: drop recovery shards beyond what the erasures need
                rec_in = list(rec)
                spare = m - len(er)
                for j in sorted(rng.choice(m, int(rng.integers(0, spare + 1)), replace=False).tolist()):
                    rec_in[j] = None
                if rng.random() < 0.15 and any(r is not None for r in rec_in):
                    j = next(i for i, r in enumerate(rec_in) if r is not None)
                    rec_in[j] = rec_in[j].copy()
                    rec_in[j][int(rng.integers(0, n))] ^= 0x5A  # corrupted, non-codeword input
                orig_in = [None if i in er else data[i] for i in range(k)]
                blocks.append((data, rec, orig_in, rec_in, er))
            with lock:
                inflight[tid] = {"case": stats["cases"], "api": api, "k": k, "m": m, "n": n,
                                 "nblocks": nblocks, "t_s": round(time.perf_counter() - t_zero, 3)}
            try:
                # encode check for every block, decode check (vs the oracle's decode of the
                # same, possibly corrupted, inputs) for blocks with erasures
                if api == "host":
                    data, rec, orig_in, rec_in, er = blocks[0]
                    got = ctx.encode(data, m)
                    ok = all(np.array_equal(g, r) for g, r in zip(got, rec))
                    if er:
                        want = oracle.decode(orig_in, rec_in, oracle.ENGINE_AVX2)
                        out = ctx.decode(orig_in, rec_in)
                        ok = ok and all(np.array_equal(out[i], want[i]) for i in want)
                elif api == "objects":
                    # the crate-shaped objects; the encoder is reused for a second
                    # round (the crate resets it once its result is released), the
                    # decoder gets its shards in random order
                    data, rec, orig_in, rec_in, er = blocks[0]
                    enc = bfrs.ReedSolomonEncoder(ctx, k, m, n)
                    ok = True
                    for rnd in range(2):
                        src = data if rnd == 0 else [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
                        want = rec if rnd == 0 else oracle.encode(src, m, oracle.ENGINE_AVX2)
                        for x in src:
                            enc.add_original_shard(x)
                        got = list(enc.encode().recovery_iter())
                        ok = ok and all(g == w.tobytes() for g, w in zip(got, want))
                    del enc
                    if er:
                        dec = bfrs.ReedSolomonDecoder(ctx, k, m, n)
                        items = [("o", i, x) for i, x in enumerate(orig_in) if x is not None] + \
                                [("r", j, x) for j, x in enumerate(rec_in) if x is not None]
                        for t_, i, x in [items[q] for q in rng.permutation(len(items))]:
                            (dec.add_original_shard if t_ == "o" else dec.add_recovery_shard)(i, x)
                        dec.decode()
                        want = oracle.decode(orig_in, rec_in, oracle.ENGINE_AVX2)
                        ok = ok and all(dec.restored_original(i) == want[i].tobytes() for i in want)
                        ok = ok and all(dec.restored_original(i) is None
                                        for i in range(k) if orig_in[i] is not None)
                        del dec
                elif api == "wrappers":
                    # generate_parity (generate.rs:59-104) with a short last segment
                    # zero-padded by the wrapper, and recover_segment_rs30_3
                    # (recovery.rs:118-173) of every erased target
                    data, rec, orig_in, rec_in, er = blocks[0]
                    cut = int(rng.integers(0, n // 2 + 1)) * 2 if k > 1 else 0
                    segs = data[:-1] + [data[-1][:n - cut]]
                    padded = data[:-1] + [np.pad(segs[-1], (0, cut))]
                    want = oracle.encode(padded, m, oracle.ENGINE_AVX2) if cut else rec
                    outs = [np.empty(n, np.uint8) for _ in range(m)]
                    bfrs.Chunker(ctx).generate_parity_into(segs, k, m, outs)
                    ok = all(np.array_equal(o, w) for o, w in zip(outs, want))
                    if k == 30 and m == 3 and er and not cut:
                        want_d = oracle.decode(orig_in, rec_in, oracle.ENGINE_AVX2)
                        if all(r is not None for r in rec_in):
                            for t in er:
                                got = bfrs.recover_segment_rs30_3(ctx, orig_in, rec_in, t)
                                ok = ok and got == want_d[t].tobytes()
                elif api == "host_batch":
                    # one shape per batch (the batch API shares k across blocks only via ks)
                    ks = [k] * nblocks
                    origs = [x for b in blocks for x in b[0]]
                    outs = [np.empty(n, np.uint8) for _ in range(m * nblocks)]
                    oi = [x for b in blocks for x in b[2]]
                    ri = [x for b in blocks for x in b[3]]
                    ro = [np.empty(n, np.uint8) if x is None else None for x in oi]
                    if rng.random() < 0.5:
                        # rows of pinned tensors at a constant pitch: the 2-D row
                        # copies of runtime.cpp copy_rows (outputs pinned too)
                        pin = torch.empty(len(origs) + len(outs) + len(oi) + len(ri) + len(ro), n,
                                          dtype=torch.uint8, pin_memory=True).numpy()
                        r0 = 0

                        def pinned(xs, fill=True):
                            nonlocal r0
                            out = []
                            for x in xs:
                                if x is None:
                                    out.append(None)
                                else:
                                    if fill:
                                        pin[r0][:] = x
                                    out.append(pin[r0])
                                r0 += 1
                            return out
                        origs = pinned(origs)
                        outs = pinned(outs, fill=False)
                        oi, ri = pinned(oi), pinned(ri)
                        ro = pinned(ro, fill=False)
                    ctx.encode_host_batch(ks, m, n, origs, outs)
                    ok = all(np.array_equal(outs[b * m + j], blocks[b][1][j])
                             for b in range(nblocks) for j in range(m))
                    ctx.decode_host_batch(ks, m, n, oi, ri, ro)
                    for b, blk in enumerate(blocks):
                        if blk[4]:
                            want = oracle.decode(blk[2], blk[3], oracle.ENGINE_AVX2)
                            ok = ok and all(np.array_equal(ro[b * k + i], want[i]) for i in want)
                else:
                    ks = [k] * nblocks
                    with torch.cuda.stream(stream):
                        d_orig = [torch.from_numpy(x).cuda() for b in blocks for x in b[0]]
                        d_rec = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(m * nblocks)]
                        ctx.encode_batch_dev(ks, m, n, d_orig, d_rec, stream=stream)
                        d_oi = [None if x is None else torch.from_numpy(x).cuda() for b in blocks for x in b[2]]
                        d_ri = [None if x is None else torch.from_numpy(x).cuda() for b in blocks for x in b[3]]
                        d_ro = [torch.empty(n, dtype=torch.uint8, device="cuda") if x is None else None
                                for x in d_oi]
                        ctx.decode_batch_dev(ks, m, n, d_oi, d_ri, d_ro, stream=stream)
                        stream.synchronize()
                    ok = all(np.array_equal(d_rec[b * m + j].cpu().numpy(), blocks[b][1][j])
                             for b in range(nblocks) for j in range(m))
                    for b, blk in enumerate(blocks):
                        if blk[4]:
                            want = oracle.decode(blk[2], blk[3], oracle.ENGINE_AVX2)
                            ok = ok and all(np.array_equal(d_ro[b * k + i].cpu().numpy(), want[i])
                                            for i in want)
            except bfrs.BfrsError as e:  # every drawn shape is valid and keeps >= k shards
                ok, err = False, f"{e.code}: {e}"
            except Exception as e:  # noqa: BLE001 -- record, keep the thread alive
                ok, err = False, f"{type(e).__name__}: {e}"
            else:
                err = None
            with lock:
                stats["cases"] += 1
                stats["bytes"] += nblocks * (k + m) * n
                stats["by_api"][api] = stats["by_api"].get(api, 0) + 1
                if not ok and not stats["failures"]:
                    stats["in_flight_at_first_failure"] = {
                        "thread": tid, "t_s": round(time.perf_counter() - t_zero, 3),
                        "threads": {str(t): dict(v) for t, v in sorted(inflight.items())}}
                if not ok and len(stats["failures"]) < 20:
                    stats["failures"].append({"api": api, "k": k, "m": m, "n": n, "nblocks": nblocks,
                                              "erasures": [b[4] for b in blocks], "error": err,
                                              "thread": tid})
                inflight.pop(tid, None)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
    for t in th:
        t.start()
    while any(t.is_alive() for t in th):  # progress on stderr (long runs must keep writing)
        th[0].join(timeout=30)
        with lock:
            print(f"progress: {stats['cases']} cases, {len(stats['failures'])} failures",
                  file=sys.stderr, flush=True)
    for t in th:
        t.join()
    ctx.close()
    stats["plan_cache"] = int(os.environ["BFRS_PLAN_CACHE"])
    stats["codec_staging"] = os.environ.get("BFRS_CODEC_STAGING", "pinned")
    stats["codec_slots"] = os.environ.get("BFRS_CODEC_SLOTS", "2")
    stats["threads"] = a.threads
    stats["huge_fraction"] = a.huge
    stats["seconds"] = a.seconds
    write_maps("at the end")
    print(json.dumps(stats))
    return 1 if stats["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
