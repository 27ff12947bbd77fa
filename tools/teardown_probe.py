"""Exit-time fault probe (measurement tool, GPU box).

Rounds 4 and 5 saw a SIGSEGV under __cxa_finalize at process exit, both
times under `rocprofv3 --kernel-trace --memory-copy-trace` (r04a bench,
r05s soak).  This program does the minimum of each kind of work and exits
normally, so the same profiler flags can be tried on less and less:

  torch  torch only: pinned and pageable H2D / D2H copies and a kernel
         (libbfrs.so is never loaded)
  bfrs   the same plus a bfrs context, a host-memory encode and decode and a
         codec object, everything closed before exit

It writes /proc/self/maps to --maps just before it returns, so the raw PCs a
fault handler prints at exit resolve to DSO + offset
(tools/resolve_pcs.py)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["torch", "bfrs"])
    ap.add_argument("--maps", default=None)
    a = ap.parse_args()
    import torch
    x = torch.arange(1 << 22, dtype=torch.int32)
    for pin in (False, True):
        h = x.pin_memory() if pin else x
        d = h.cuda()
        d.mul_(3)
        back = d.cpu()
        assert int(back[7]) == 21
    torch.cuda.synchronize()
    if a.mode == "bfrs":
        import numpy as np
        sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
        import bfrs
        ctx = bfrs.Context(0)
        rng = np.random.default_rng(3)
        shards = [rng.integers(0, 256, 1 << 20, dtype=np.uint8) for _ in range(30)]
        rec = ctx.encode(shards, 3)
        out = ctx.decode([None, None, None] + shards[3:], rec)
        assert all(np.array_equal(out[i], shards[i]) for i in range(3))
        enc = bfrs.ReedSolomonEncoder(ctx, 30, 3, 1 << 20)
        for s in shards:
            enc.add_original_shard(s)
        enc.encode()
        assert bytes(enc.recovery_view(1)) == rec[1].tobytes()
        enc.free()
        ctx.close()
    if a.maps:
        with open("/proc/self/maps") as f, open(a.maps, "w") as o:
            o.write(f.read())
    print(f"teardown_probe {a.mode}: work done, exiting normally", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
