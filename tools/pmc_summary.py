"""Per-launch HBM traffic of gf_apply from rocprofv3 PMC passes.

usage: python tools/pmc_summary.py gpurun_out/prof_TAG [TAG [BOX]] > profiles/pmc_traffic.json

Reads <dir>_FETCH_SIZE/pmc_counter_collection.csv and <dir>_WRITE_SIZE/...
(separate --pmc passes of the bench command), keeps the full-size gf_apply
dispatches (the C2 launches: > 1M threads), and applies the gfx950
corrections of MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB and
FETCH_SIZE counts half of a 16 B/lane streaming read (x2)."""
import csv
import json
import os
import statistics
import sys


C2_GRID = 20480 * 256  # 4 x RS(30,3) + 1 x RS(8,3) of 32 MiB: 8 KiB tiles, 256 lanes


def values(path, counter):
    """Per-dispatch counter value (summed over its dimension rows) of the C2
    launches (the bench's value; C4 and small launches have other grids)."""
    per = {}
    for r in csv.DictReader(open(path)):
        if "gf_apply" in r["Kernel_Name"] and r["Counter_Name"] == counter \
                and int(r["Grid_Size"]) == C2_GRID:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(per.values())


def trace_ms(path):
    """Launch durations (ms) of the C2 launches in the --kernel-trace pass."""
    if not os.path.exists(path):
        return None
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
         for r in csv.DictReader(open(path))
         if "gf_apply" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == C2_GRID]
    return {"launches": len(d), "mean_ms": round(statistics.mean(d), 4),
            "median_ms": round(statistics.median(d), 4), "min_ms": round(min(d), 4),
            "max_ms": round(max(d), 4), "file": "run_kernel_trace.csv (--kernel-trace --stats pass)"}


def main():
    base = sys.argv[1].rstrip("/")
    tag = sys.argv[2] if len(sys.argv) > 2 else base.rsplit("_", 1)[-1]
    box = sys.argv[3] if len(sys.argv) > 3 else None
    f = values(base + "_FETCH_SIZE/pmc_counter_collection.csv", "FETCH_SIZE")
    w = values(base + "_WRITE_SIZE/pmc_counter_collection.csv", "WRITE_SIZE")
    fk, wk = statistics.median(f), statistics.median(w)
    rd, wr = int(fk * 1024 * 2), int(wk * 1024)
    alg_r, alg_w = 128 * 32 << 20, 15 * 32 << 20
    kernel = next(r["Kernel_Name"] for r in csv.DictReader(
        open(base + "_FETCH_SIZE/pmc_counter_collection.csv"))
        if "gf_apply" in r["Kernel_Name"] and int(r["Grid_Size"]) == C2_GRID)
    print(json.dumps({
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of the "
                  f"driver's bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5), "
                  f"{tag}",
        "round": tag, "box": box,
        "kernel": kernel.replace("void ", "").split("(bfrs::KernArgs)")[0],
        "grid": C2_GRID,
        "dispatches": len(f),
        "correction": "FETCH_SIZE and WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half of a "
                      "16 B/lane streaming read (MI355X_MICROARCH.md HBM section) -> x2",
        "fetch_size_kib_median": fk, "write_size_kib_median": wk,
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "algorithmic_read_bytes": alg_r, "algorithmic_write_bytes": alg_w,
        "ratio_to_algorithmic": round((rd + wr) / (alg_r + alg_w), 4),
        "trace": trace_ms(base + "/run_kernel_trace.csv"),
    }, indent=1))


if __name__ == "__main__":
    main()
