"""Same-process A/B of a device BLAKE3 variant of the measurement build, read
per call from the environment: round 4's kernel-1 tree depth
(BFRS_B3_GROUP_LEVELS = 2 / 3, since removed) and now kernel 2's quad levels
(AB_VAR=BFRS_B3_QUADS, values 1 / 0, the default).  C2's 128 x 32 MiB
HBM-resident segments, alternating variants, best and median wall time per
call and the group / reduce kernel times from torch's profiler.  Loads the
measurement build (make -C blockframe-rs_amd/csrc ab -> libbfrs_ab.so,
BFRS_LIB).  GPU box only."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
import bfrs  # noqa: E402


def kernel_ms(ctx, segs, calls=3):
    from torch.autograd import DeviceType
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(calls):
            ctx.blake3_batch_dev(segs)
    ev = [(e.name(), e.duration_ns() / 1e6) for e in prof.profiler.kineto_results.events()
          if e.device_type() == DeviceType.CUDA and "blake3" in e.name()]
    return (round(statistics.median(d for n, d in ev if "group" in n), 4),
            round(sum(d for n, d in ev if "reduce" in n) / calls, 4))


def main():
    S, nseg, rounds = 32 << 20, 128, int(os.environ.get("AB_ROUNDS", "4"))
    ctx = bfrs.Context(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    buf = torch.randint(0, 256, (nseg * S,), dtype=torch.uint8, device="cuda", generator=g)
    segs = [buf[i * S:(i + 1) * S] for i in range(nseg)]
    var = os.environ.get("AB_VAR", "BFRS_B3_QUADS")
    va, vb = os.environ.get("AB_VALUES", "1,0").split(",")
    res = {va: [], vb: []}
    kern = {va: [], vb: []}
    digests = {}
    for r in range(rounds):
        for lv in ((va, vb) if r % 2 == 0 else (vb, va)):
            os.environ[var] = lv
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:  # settle
                ctx.blake3_batch_dev(segs)
            for _ in range(10):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                d = ctx.blake3_batch_dev(segs)
                res[lv].append(time.perf_counter() - t1)
            digests[lv] = d
            kern[lv].append(kernel_ms(ctx, segs))
    assert digests[va] == digests[vb]
    out = {"what": f"device BLAKE3 of 128 x 32 MiB, {var} = {va} vs {vb}, alternated in one "
                   "process (tools/b3_levels_ab.py, measurement build)", "digests_equal": True}
    for lv in (va, vb):
        ts = res[lv]
        out[lv] = {"best_ms": round(min(ts) * 1e3, 4), "median_ms": round(statistics.median(ts) * 1e3, 4),
                   "GBps_best": round(nseg * S / min(ts) / 1e9, 1),
                   "group_kernel_ms": [k[0] for k in kern[lv]],
                   "reduce_ms": [k[1] for k in kern[lv]]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
