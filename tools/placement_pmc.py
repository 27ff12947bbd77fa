"""Placement study under PMC: C copies of the bench's separate-set layout
(128 data rows + 15 parity rows each), encoded L times per copy in a fixed
order, so that a `rocprofv3 --pmc ...` run of this script gives every
copy's launches in sequence (dispatch order = copy-major).  Run it under the
profiler, then `--summarize` the counter CSV: per copy, the median launch
duration (from the PMC record's timestamps) and the median of each counter,
i.e. what differs between a fast and a slow placement in ONE process.

usage: rocprofv3 --pmc A B -d DIR -o pmc -- python3 tools/placement_pmc.py [--copies 6] [--launches 20]
       python3 tools/placement_pmc.py --summarize DIR/pmc_counter_collection.csv [--copies 6] [--launches 20]
"""
import argparse
import collections
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "blockframe-rs_amd"))
C2_GRID = 20480 * 256


def run(a):
    import torch
    import bfrs
    from bfrs import synth
    S = synth.SEGMENT_SIZE
    shapes = synth.block_shapes(128)
    nb = len(shapes)
    pitch = bfrs.shard_pitch(S)

    flats = []

    def rows(n):
        buf = torch.empty(n * pitch, dtype=torch.uint8, device="cuda")
        flats.append(buf)
        return [buf[i * pitch:i * pitch + S] for i in range(n)]

    copies = []
    for _ in range(a.copies):
        d = rows(128)
        for s_ in range(128):
            synth.fill_segment_torch(d[s_], 0xB10C, s_)
        copies.append((d, rows(3 * nb)))
    ctx = bfrs.Context(0)
    stream = torch.cuda.current_stream()
    # clock settle (the first ~30 launches after an idle gap ramp):
    # launches of the last copy, dropped by --summarize
    for _ in range(a.settle):
        ctx.encode_batch_dev(shapes, 3, S, copies[-1][0], copies[-1][1], stream=stream)
    timing = []
    for c, (d, p) in enumerate(copies):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record(stream)
        for _ in range(a.launches):
            ctx.encode_batch_dev(shapes, 3, S, d, p, stream=stream)
        e[1].record(stream)
        torch.cuda.synchronize()
        row = {"copy": c, "encode_ms": round(e[0].elapsed_time(e[1]) / a.launches, 4)}
        if a.probe:  # plain streams over the same data allocation, settled the same way
            flat = flats[2 * c]
            h = flat.numel() // 2
            import ctypes
            sp = ctypes.CDLL(os.path.join(ROOT, "tools", "libstreamprobe.so"))
            scratch = torch.empty(1 << 20, dtype=torch.int64, device="cuda")
            sh = ctypes.c_void_p(stream.cuda_stream)
            nt_read = lambda: sp.bfrs_probe_read(ctypes.c_void_p(flat.data_ptr()),  # noqa: E731
                                                 ctypes.c_size_t(flat.numel()),
                                                 ctypes.c_void_p(scratch.data_ptr()), sh)
            nt_write = lambda: sp.bfrs_probe_write(ctypes.c_void_p(flat.data_ptr()),  # noqa: E731
                                                   ctypes.c_size_t(flat.numel()), sh)
            for name, fn in (("copy", lambda: flat[h:2 * h].copy_(flat[:h])),
                             ("read", lambda: flat.view(torch.int64).sum()),
                             ("fill", lambda: flat.fill_(7)),
                             ("ntread", nt_read), ("ntwrite", nt_write)):
                for _ in range(10):
                    fn()
                e[0].record(stream)
                for _ in range(a.launches):
                    fn()
                e[1].record(stream)
                torch.cuda.synchronize()
                ms = e[0].elapsed_time(e[1]) / a.launches
                nbytes = 2 * h if name == "copy" else flat.numel()
                row[f"{name}_GBps"] = round(nbytes / ms / 1e6, 1)
        timing.append(row)
    print(json.dumps({"copies": a.copies, "launches": a.launches, "timing": timing,
                      "addresses": [hex(d[0].data_ptr()) for d, _ in copies]}, indent=1))


def pitch_sweep(a):
    """Row pitch vs placement: every pitch runs inside the same allocation
    of each copy, so a pitch that is fast in a slow copy is a layout fix."""
    import torch
    import bfrs
    from bfrs import synth
    S = synth.SEGMENT_SIZE
    shapes = synth.block_shapes(128)
    nb = len(shapes)
    extras = [int(x) for x in a.pitches.split(",")]
    big = S + max(extras)
    bufs = [torch.empty(143 * big, dtype=torch.uint8, device="cuda") for _ in range(a.copies)]
    ctx = bfrs.Context(0)
    stream = torch.cuda.current_stream()
    layouts = {}
    for c, buf in enumerate(bufs):
        for x in extras:
            pitch = S + x
            r = [buf[i * pitch:i * pitch + S] for i in range(143)]
            layouts[(c, x)] = (r[:128], r[128:128 + 3 * nb])
    for c in range(a.copies):  # data bytes once per copy (rows of every pitch overlap)
        d, _ = layouts[(c, extras[0])]
        for s_ in range(128):
            synth.fill_segment_torch(d[s_], 0xB10C, s_)
    for _ in range(a.settle):
        ctx.encode_batch_dev(shapes, 3, S, *layouts[(0, extras[0])], stream=stream)
    res = {}
    import random
    order = list(layouts)
    random.Random(7).shuffle(order)
    for key in order:
        d, p = layouts[key]
        for _ in range(5):
            ctx.encode_batch_dev(shapes, 3, S, d, p, stream=stream)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record(stream)
        for _ in range(a.launches):
            ctx.encode_batch_dev(shapes, 3, S, d, p, stream=stream)
        e[1].record(stream)
        torch.cuda.synchronize()
        res[key] = round(e[0].elapsed_time(e[1]) / a.launches, 4)
    print(json.dumps({"pitch_extra_bytes": extras,
                      "encode_ms": {f"copy{c}": [res[(c, x)] for x in extras] for c in range(a.copies)},
                      "addresses": [hex(b.data_ptr()) for b in bufs]}, indent=1))


def cross(a):
    """Encode D_i -> P_j for every pair of copies: does a slow placement
    follow the data rows (reads) or the parity rows (writes)?"""
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

    D, P = [], []
    for _ in range(a.copies):
        d = rows(128)
        for s_ in range(128):
            synth.fill_segment_torch(d[s_], 0xB10C, s_)
        D.append(d)
        P.append(rows(3 * nb))
    ctx = bfrs.Context(0)
    stream = torch.cuda.current_stream()
    for _ in range(a.settle):
        ctx.encode_batch_dev(shapes, 3, S, D[0], P[0], stream=stream)
    ms = [[0.0] * a.copies for _ in range(a.copies)]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for i in range(a.copies):
        for j in range(a.copies):
            for _ in range(3):
                ctx.encode_batch_dev(shapes, 3, S, D[i], P[j], stream=stream)
            e[0].record(stream)
            for _ in range(a.launches):
                ctx.encode_batch_dev(shapes, 3, S, D[i], P[j], stream=stream)
            e[1].record(stream)
            torch.cuda.synchronize()
            ms[i][j] = round(e[0].elapsed_time(e[1]) / a.launches, 4)
    print(json.dumps({"encode_ms_data_i_parity_j": ms,
                      "data": [hex(d[0].data_ptr()) for d in D],
                      "parity": [hex(p[0].data_ptr()) for p in P]}, indent=1))


def summarize(a):
    per = collections.defaultdict(dict)  # dispatch -> {counter: value, "ns": duration}
    inst = collections.defaultdict(lambda: collections.defaultdict(list))  # dispatch -> counter -> rows
    for r in csv.DictReader(open(a.summarize)):
        if "gf_apply" not in r["Kernel_Name"] or int(r["Grid_Size"]) != C2_GRID:
            continue
        d = per[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        inst[int(r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if a.instances:  # spread of a counter over its hardware instances (e.g. TCC channels)
        ids = sorted(per)[-a.copies * a.launches:]
        out = []
        for c in range(a.copies):
            sel = ids[c * a.launches:(c + 1) * a.launches][3:]
            if not sel:
                continue
            row = {"copy": c, "ms": round(statistics.median(per[i]["ns"] for i in sel) / 1e6, 4)}
            for k in sorted(inst[sel[0]]):
                vals = [inst[i][k] for i in sel]
                n = len(vals[0])
                mean_inst = [statistics.mean(v[j] for v in vals) for j in range(n)]
                m = statistics.mean(mean_inst)
                row[k] = {"instances": n, "sum": round(sum(mean_inst), 1),
                          "max_over_mean": round(max(mean_inst) / m, 4) if m else None,
                          "min_over_mean": round(min(mean_inst) / m, 4) if m else None,
                          "cv": round(statistics.pstdev(mean_inst) / m, 4) if m and n > 1 else None,
                          "per_instance": [round(x, 1) for x in mean_inst] if n <= 128 else None}
            out.append(row)
        print(json.dumps(out, indent=1))
        return
    ids = sorted(per)[-a.copies * a.launches:]  # after the settle launches
    out = []
    for c in range(a.copies):
        ds = [per[i] for i in ids[c * a.launches:(c + 1) * a.launches]][3:]  # skip ramp
        if not ds:
            continue
        keys = sorted(k for k in ds[0] if k != "ns")
        out.append({"copy": c, "ms": round(statistics.median(x["ns"] for x in ds) / 1e6, 4),
                    **{k: statistics.median(x[k] for x in ds) for k in keys}})
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=6)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--settle", type=int, default=60, help="untimed launches before the copies")
    ap.add_argument("--summarize", default=None)
    ap.add_argument("--instances", action="store_true",
                    help="with --summarize: each counter's spread over its hardware instances")
    ap.add_argument("--pitches", default=None,
                    help="comma list of row pitches minus S (bytes): per copy, one buffer of 143 rows at "
                         "the largest pitch, encode timed with each pitch inside the same buffer")
    ap.add_argument("--cross", action="store_true", help="encode D_i -> P_j for every pair")
    ap.add_argument("--probe", action="store_true",
                    help="also time a torch copy / read / fill over each copy's data allocation")
    a = ap.parse_args()
    if a.summarize:
        summarize(a)
    elif a.cross:
        cross(a)
    elif a.pitches:
        pitch_sweep(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
