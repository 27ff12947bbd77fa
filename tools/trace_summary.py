"""C2 launch summary of a rocprofv3 --kernel-trace --stats run of the bench.

usage: python tools/trace_summary.py gpurun_out/prof_TAG [STEPS] > c2_launch_summary.json

Reads the run's *kernel_trace.csv and *kernel_stats.csv (found anywhere under
the directory), keeps the gf_apply dispatches at the C2 grid (4 x RS(30,3) +
1 x RS(8,3) of 32 MiB: 20,480 workgroups of 256 lanes; config 4, the slab
pipelines and the tests' launches have other grids) and reports their
duration statistics, the --stats line of the kernel, and the profiled bench
line's own launch_ms (bench_under_rocprof.json beside the trace, if present)
with the ratio of the trace mean to it."""
import csv
import glob
import json
import os
import statistics
import sys

C2_GRID = 20480 * 256


def main():
    base = sys.argv[1].rstrip("/")
    traces = glob.glob(os.path.join(base, "**", "*kernel_trace.csv"), recursive=True)
    stats = glob.glob(os.path.join(base, "**", "*kernel_stats.csv"), recursive=True)
    if not traces:
        sys.exit(f"no kernel_trace.csv under {base}")
    rows = [r for t in traces for r in csv.DictReader(open(t))
            if "gf_apply" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == C2_GRID]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    if not d:
        sys.exit("no C2-grid gf_apply dispatches in the trace")
    steady = d[64:] if len(d) > 128 else d  # past the clock ramp of the first launches
    out = {"kernel": rows[0]["Kernel_Name"].replace("void ", "").split("(bfrs::KernArgs)")[0],
           "grid": C2_GRID, "launches": len(d),
           "mean_ms": round(statistics.mean(d), 4), "median_ms": round(statistics.median(d), 4),
           "min_ms": round(min(d), 4), "max_ms": round(max(d), 4),
           "mean_ms_after_first_64": round(statistics.mean(steady), 4),
           "alg_bytes_per_launch": 143 * (32 << 20),
           "frac_at_mean": round(143 * (32 << 20) / (statistics.mean(d) * 1e-3) / 8e12, 4)}
    for st in stats:
        for r in csv.DictReader(open(st)):
            if "gf_apply_unrolled" in r["Name"]:
                out["stats_gf_apply_unrolled"] = {"calls": int(r["Calls"]),
                                                  "average_ms": round(float(r["AverageNs"]) / 1e6, 4),
                                                  "percentage": float(r["Percentage"])}
    line_path = os.path.join(base, "bench_under_rocprof.json")
    if os.path.exists(line_path):
        try:
            lines = [l for l in open(line_path) if l.startswith("{")]
            line = json.loads(lines[-1])
            lm = line["roofline"]["launch_ms"]
            out["bench_line_launch_ms"] = lm
            out["ratio_mean_to_line_launch_ms"] = round(out["mean_ms"] / lm, 4)
            out["ratio_steady_mean_to_line_launch_ms"] = round(out["mean_ms_after_first_64"] / lm, 4)
        except (OSError, ValueError, KeyError, IndexError) as e:
            out["bench_line_error"] = f"{type(e).__name__}: {e}"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
