"""How fast is BlockFrame's own call pattern on the crate-shaped path?

commit_blocked runs Chunker::generate_parity once per block from rayon
workers (src/chunker/commit.rs:391-466), every block's segments new mmap'd
pages.  This probe runs C2's blocks (30+30+30+30+8 x 32 MiB) on as many
threads sharing one context, per BFRS_CODEC_STAGING mode:
  seen_<mode>   the same input buffers every round (HIP has seen them)
  fresh_<mode>  new input buffers every round (copied untimed), as BlockFrame
Outputs are fresh np.empty buffers every round (the reference's to_vec()).
Also the box's link floor for the batch (H2D of all inputs + D2H of all
parity, torch copies from/to pinned memory).  Prints one JSON line.
GPU box only (tools/, not a test)."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "blockframe-rs_amd"))
os.environ.setdefault("BFRS_CODEC_SLOTS", "8")
import numpy as np  # noqa: E402
import bfrs  # noqa: E402

S = 32 << 20
SHAPES = [int(x) for x in os.environ.get("PROBE_SHAPES", "30,30,30,30,8").split(",")]
REPS = int(os.environ.get("PROBE_REPS", "4"))


def context(mode):
    old = os.environ.get("BFRS_CODEC_STAGING")
    os.environ["BFRS_CODEC_STAGING"] = mode
    try:
        return bfrs.Context(0)
    finally:
        if old is None:
            del os.environ["BFRS_CODEC_STAGING"]
        else:
            os.environ["BFRS_CODEC_STAGING"] = old


def run_blocks(ctx, blocks):
    errors = []

    def worker(b):
        try:
            bfrs.Chunker(ctx).generate_parity_into(
                blocks[b], len(blocks[b]), 3, [np.empty(S, np.uint8) for _ in range(3)])
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
    ts = [threading.Thread(target=worker, args=(b,)) for b in range(len(blocks))]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    el = time.perf_counter() - t0
    assert not errors, errors
    return el


def cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def main():
    node = os.environ.get("PROBE_NODE")
    if node is not None:  # this process (and every thread it starts) on one NUMA node's CPUs
        os.sched_setaffinity(0, cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read()))
    import torch
    if os.environ.get("PROBE_PINNED_GIB"):  # torch pinned memory allocated and freed first (bench's pcie_inclusive)
        t = torch.empty(int(float(os.environ["PROBE_PINNED_GIB"]) * 2**30), dtype=torch.uint8,
                        pin_memory=True)
        t.fill_(1)
        del t
    rng = np.random.default_rng(3)
    base = rng.integers(0, 256, S, dtype=np.uint8)
    blocks = [[np.roll(base, 64 * (b * 31 + i)) for i in range(k)] for b, k in enumerate(SHAPES)]
    if os.environ.get("PROBE_TORCH_SEGS"):  # segments as bench.py makes them: .cpu() of device rows
        dev = torch.from_numpy(np.stack([x for blk in blocks for x in blk])).cuda()
        it = iter(range(sum(SHAPES)))
        blocks = [[dev[next(it)].cpu().numpy() for _ in range(k)] for k in SHAPES]
        del dev
    if os.environ.get("PROBE_GPU_WORK"):  # seconds of HBM-bound device copies first, as bench.py's kernel run
        a = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < float(os.environ["PROBE_GPU_WORK"]):
            for _ in range(20):
                b.copy_(a)
            torch.cuda.synchronize()
        if os.environ.get("PROBE_KEEP_HBM") is None:
            del a, b
    gib = sum(SHAPES) * S / 2**30
    res = {"what": f"blocks {SHAPES} x {S >> 20} MiB on {len(SHAPES)} threads, one context; "
                   f"ms (best, median of {REPS})", "host_copy_threads": os.environ.get(
                       "BFRS_HOST_COPY_THREADS", "default"),
           "torch_segs": bool(os.environ.get("PROBE_TORCH_SEGS")),
           "pinned_gib_first": os.environ.get("PROBE_PINNED_GIB"),
           "gpu_work_s_first": os.environ.get("PROBE_GPU_WORK"),
           "numa_node_cpus": node}
    n_in, n_out = sum(SHAPES) * S, 3 * len(SHAPES) * S
    dev = torch.empty(n_in, dtype=torch.uint8, device="cuda")
    pin = torch.empty(n_in, dtype=torch.uint8, pin_memory=True)
    pin.fill_(1)

    def xfer():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dev.copy_(pin, non_blocking=True)
        pin[:n_out].copy_(dev[:n_out], non_blocking=True)
        torch.cuda.synchronize()
        return time.perf_counter() - t0
    res["link_floor_ms"] = round(min(xfer() for _ in range(3)) * 1e3, 2)
    del dev, pin
    for mode in os.environ.get("PROBE_MODES", "pinned,direct").split(","):
        ctx = context(mode)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:  # link settle
            run_blocks(ctx, blocks)
        seen = [run_blocks(ctx, blocks) for _ in range(REPS)]
        fresh = []
        for _ in range(REPS):
            nb = [[np.array(x) for x in blk] for blk in blocks]
            fresh.append(run_blocks(ctx, nb))
            del nb
        for key, ts in ((f"seen_{mode}", seen), (f"fresh_{mode}", fresh)):
            res[key] = [round(min(ts) * 1e3, 2), round(float(np.median(ts)) * 1e3, 2)]
            res[key + "_GiBps"] = round(gib / min(ts), 2)
        ctx.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
