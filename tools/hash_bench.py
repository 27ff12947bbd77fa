"""Device BLAKE3 throughput: 128 x 32 MiB HBM-resident segments per call
(what a 4 GiB tier-3 commit hashes), timed over K calls.  Each call includes
the descriptor upload, both kernels and the 4 KiB digest download."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
import bfrs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=128)
    ap.add_argument("--segment-bytes", type=int, default=32 << 20)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    ctx = bfrs.Context(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    buf = torch.randint(0, 256, (args.segments * args.segment_bytes,), dtype=torch.uint8,
                        device="cuda", generator=g)
    segs = [buf[i * args.segment_bytes:(i + 1) * args.segment_bytes] for i in range(args.segments)]
    for _ in range(3):
        ctx.blake3_batch_dev(segs)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        ctx.blake3_batch_dev(segs)
    dt = (time.perf_counter() - t) / args.steps
    nbytes = args.segments * args.segment_bytes
    print(json.dumps({"metric": "device BLAKE3 GB/s", "value": round(nbytes / dt / 1e9, 1),
                      "ms_per_call": round(dt * 1e3, 3), "segments": args.segments,
                      "segment_bytes": args.segment_bytes}))


if __name__ == "__main__":
    main()
