#!/bin/bash
# Round-6 GPU-box session: the driver argv, its rocprofv3 kernel trace, the GPU suite and smoke.
#  1. The driver's bench command VERBATIM: python3 bench.py --gpus 1 --steps 20 --warmup 5
#     (the line goes to gpurun_out/bench_$TAG.json, stderr beside it).
#  2. The same argv under rocprofv3 --kernel-trace --stats (the profiled process
#     is the measurement: no supervisor, no child passes under the profiler),
#     summarised by tools/pmc_summary.py-style C2 launch stats.
#  3. Optionally the -m gpu suite and smoke (SUITE=1).
# Every GPU step has its own time limit; any failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r06}
export TMPDIR=/tmp
hostname > "$OUT/box_$TAG.txt"

if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
      > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench_$TAG.err"
  [ $rc -eq 0 ] || exit $rc
fi

if [ "${SKIP_PROF:-0}" != 1 ]; then
  mkdir -p "$OUT/prof_$TAG"
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$OUT/prof_$TAG" -o run -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 \
      > "$OUT/prof_$TAG/bench_under_rocprof.json" 2> "$OUT/prof_$TAG/bench_under_rocprof.err"
  rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/trace_summary.py "$OUT/prof_$TAG" 20 > "$OUT/prof_$TAG/c2_launch_summary.json"
  rc=$?; echo "summary rc=$rc"; [ $rc -eq 0 ] || exit $rc
  # keep the stats and the summary, not the multi-MB trace
  find "$OUT/prof_$TAG" -name '*kernel_trace.csv' -delete
fi

if [ "${SUITE:-0}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; tail -2 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi
echo "r06_check done"
