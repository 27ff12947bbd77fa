"""Placement study: is a slow launch a property of the read rows or of where
the outputs land?  One data set D is encoded into several separately
allocated parity sets P_i (and a second data set D2 into P_0), each timed
like tools/kbench.py (settled, HIP events, median of rounds).  Encode timing
only; outputs are checked against the first parity set at the end.

usage: python tools/placement_probe.py [--outputs 6] [--rounds 3] [--iters 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--outputs", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--settle-ms", type=float, default=200.0)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bfrs
    from bfrs import synth
    S = synth.SEGMENT_SIZE
    shapes = synth.block_shapes(128)
    nb = len(shapes)
    pitch = bfrs.shard_pitch(S)

    def rows(n):
        buf = torch.empty(n * pitch, dtype=torch.uint8, device="cuda")
        return [buf[i * pitch:i * pitch + S] for i in range(n)]

    D = rows(128)
    for s_ in range(128):
        synth.fill_segment_torch(D[s_], 0xB10C, s_)
    outs = [rows(3 * nb) for _ in range(a.outputs)]
    D2 = rows(128)
    for s_ in range(128):
        synth.fill_segment_torch(D2[s_], 0xB10C, s_)
    cases = {f"D->P{i}": (D, outs[i]) for i in range(a.outputs)}
    cases["D2->P0"] = (D2, outs[0])
    ctx = bfrs.Context(0)
    stream = torch.cuda.current_stream()
    alg = sum(k + 3 for k in shapes) * S

    def run(c):
        src, dst = cases[c]
        ctx.encode_batch_dev(shapes, 3, S, src, dst, stream=stream)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        run("D->P0")
    torch.cuda.synchronize()
    res = {c: [] for c in cases}
    import random
    rng = random.Random(0x5EED)
    for _ in range(a.rounds):
        order = list(cases)
        rng.shuffle(order)
        for c in order:
            t1 = time.perf_counter()
            while time.perf_counter() - t1 < a.settle_ms / 1e3:
                run(c)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.iters):
                run(c)
            e1.record(stream)
            torch.cuda.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.iters)
    ref = torch.stack(outs[0])
    for i in range(1, a.outputs):
        assert torch.equal(torch.stack(outs[i]), ref), f"P{i} differs"
    out = {c: {"ms": round(float(np.median(v)), 4), "GBps": round(alg / float(np.median(v)) / 1e6, 1),
               "all_ms": [round(x, 4) for x in v]} for c, v in res.items()}
    out["addresses"] = {"D": hex(D[0].data_ptr()), "D2": hex(D2[0].data_ptr()),
                        **{f"P{i}": hex(o[0].data_ptr()) for i, o in enumerate(outs)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
