import os, sys, time, tempfile, numpy as np
sys.path.insert(0, "blockframe-rs_amd")
import bfrs
t=time.perf_counter(); ctx = bfrs.Context(0); print("open", round(time.perf_counter()-t,4))
work = tempfile.mkdtemp()
for i in range(3):
    src = os.path.join(work, f"f{i}.bin")
    open(src, "wb").write(np.random.default_rng(i).integers(0, 256, 24_000_000, dtype=np.uint8).tobytes())
    t = time.perf_counter(); bfrs.commit(ctx, src, os.path.join(work, f"a{i}")); dt = time.perf_counter() - t
    print("tier1 commit", i, round(dt, 4), "s", round(24e6/dt/1e6,1), "MB/s")
src = os.path.join(work, "g.bin")
open(src, "wb").write(np.random.default_rng(9).integers(0, 256, 200_000_000, dtype=np.uint8).tobytes())
for i in range(2):
    t = time.perf_counter(); bfrs.commit(ctx, src, os.path.join(work, f"b{i}")); dt = time.perf_counter() - t
    print("tier2 commit 200MB", i, round(dt, 4), "s", round(200e6/dt/1e6,1), "MB/s")
