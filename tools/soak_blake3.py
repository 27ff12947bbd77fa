"""GPU soak of the device BLAKE3 (blake3_kernels.hip), the oracle as checker.

For a fixed wall time: random batches of device messages whose lengths are
drawn around every tree boundary (1 KiB chunks, 64-B blocks, 256 KiB kernel-1
groups, multi-level reductions), digests compared with oracle/blake3_oracle.c;
and random files split into power-of-two segments hashed at their chunk
offsets, the file hash rebuilt with bfrs_blake3_combine (the commit path's
whole-file hash, commit.rs:478).  Prints one JSON line; exit 1 on any mismatch.

usage: python3 tools/soak_blake3.py [--seconds 60]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--seed", type=int, default=0xB1A3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bfrs
    import oracle

    ctx = bfrs.Context(0)
    rng = np.random.default_rng(a.seed)
    K, G = 1024, 256 * 1024
    bases = [0, 1, 63, 64, 65, K - 1, K, K + 1, G - 1, G, G + 1, 2 * G, 7 * G + 3, 1 << 20]
    st = {"messages": 0, "bytes": 0, "combines": 0, "failures": []}
    stop = time.perf_counter() + a.seconds
    last = time.perf_counter()
    while time.perf_counter() < stop:
        if rng.random() < 0.7:
            n = int(rng.integers(1, 17))
            lens = []
            for _ in range(n):
                b = int(rng.choice(bases + [int(rng.integers(0, 4 << 20))]))
                lens.append(max(0, b + int(rng.integers(-2, 3))))
            host = [rng.integers(0, 256, l, dtype=np.uint8) for l in lens]
            dev = [torch.from_numpy(h).cuda() if h.size else torch.empty(0, dtype=torch.uint8, device="cuda")
                   for h in host]
            got = ctx.blake3_batch_dev(dev)
            for h, g in zip(host, got):
                if g != oracle.blake3_hex(h) and len(st["failures"]) < 20:
                    st["failures"].append({"kind": "digest", "len": int(h.size)})
            st["messages"] += n
            st["bytes"] += int(sum(lens))
        else:
            part = int(rng.choice([K, 4 * K, G, 1 << 20]))  # power-of-two segment sizes
            nseg = int(rng.integers(2, 9))
            size = (nseg - 1) * part + int(rng.integers(1, part + 1))
            data = rng.integers(0, 256, size, dtype=np.uint8)
            d = torch.from_numpy(data).cuda()
            segs = [d[i:i + part] for i in range(0, size, part)]
            offs = [i * (part // K) for i in range(len(segs))]
            _, cvs = ctx.blake3_batch_dev(segs, with_cvs=True, chunk_offsets=offs)
            if bfrs.blake3_combine(cvs) != oracle.blake3_hex(data) and len(st["failures"]) < 20:
                st["failures"].append({"kind": "combine", "size": size, "part": part})
            st["combines"] += 1
            st["bytes"] += size
        if time.perf_counter() - last > 30:  # progress on stderr (long runs must keep writing)
            last = time.perf_counter()
            print(f"progress: {st['messages']} messages, {st['combines']} combines", file=sys.stderr, flush=True)
    ctx.close()
    st["seconds"] = a.seconds
    print(json.dumps(st))
    return 1 if st["failures"] else 0


if __name__ == "__main__":
    sys.exit(main())
