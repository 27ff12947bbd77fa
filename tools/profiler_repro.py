"""Round 4's SIGSEGV suspect, in isolation (GPU box; diagnostic only).

Round 4's driver run died by SIGSEGV in the bench's blake3_device leg, the leg
that opened a SECOND in-process torch.profiler session (kineto over the ROCm
tracer) after a first one that had logged "ROCTracer produced duplicate flow
start" (DESIGN.md §5).  This probe repeats that sequence without the bench:
session 1 traces settle launches + 40 gf_apply launches of a C2-shaped batch
through libbfrs.so, then bfrs_blake3_batch_dev calls run untraced, then
session 2 traces 3 more BLAKE3 calls; the pair repeats `--rounds` times in
one process.  faulthandler prints the stack of a crash; otherwise one JSON
line says how many session pairs completed.  (The bench itself runs no
profiler since round 5.)"""
import argparse
import faulthandler
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))


def main():
    faulthandler.enable(all_threads=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--segments", type=int, default=128)
    ap.add_argument("--segment-bytes", type=int, default=32 << 20)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile
    import bfrs
    from bfrs import synth
    shapes = synth.block_shapes(a.segments)
    S = a.segment_bytes
    nseg, nb = sum(shapes), len(shapes)
    data = torch.empty(nseg, S, dtype=torch.uint8, device="cuda")
    for s in range(nseg):
        synth.fill_segment_torch(data[s], 0xB10C, s)
    par = torch.empty(3 * nb, S, dtype=torch.uint8, device="cuda")
    ctx = bfrs.Context(0)
    enc = ctx.prepare_encode(shapes, 3, S, [data[s] for s in range(nseg)],
                             [par[i] for i in range(3 * nb)])
    sh = torch.cuda.current_stream().cuda_stream
    rows = [data[s] for s in range(nseg)]
    call, dig = ctx.blake3_batch_dev_call(rows)
    done, events = 0, []
    t0 = time.perf_counter()
    for r in range(a.rounds):
        with profile(activities=[ProfilerActivity.CUDA]) as p1:
            t = time.perf_counter()
            while time.perf_counter() - t < 0.3:
                enc(sh)
            for _ in range(40):
                enc(sh)
            torch.cuda.synchronize()
        n1 = sum(1 for e in p1.profiler.kineto_results.events() if "gf_apply" in e.name())
        for _ in range(10):
            call()
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as p2:
            for _ in range(3):
                call()
            torch.cuda.synchronize()
        n2 = sum(1 for e in p2.profiler.kineto_results.events() if "blake3" in e.name())
        events.append([n1, n2])
        done += 1
        print(f"round {r}: session pair done ({n1} gf_apply, {n2} blake3 events)",
              file=sys.stderr, flush=True)
    ctx.close()
    print(json.dumps({"session_pairs_completed": done, "events": events,
                      "seconds": round(time.perf_counter() - t0, 1),
                      "digest0": bytes(dig[0]).hex()}))


if __name__ == "__main__":
    main()
