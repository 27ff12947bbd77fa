#!/bin/bash
# Round-4 GPU-box session: the driver's default bench command (with the live
# kernel-trace pass kept under gpurun_out/$TAG_prof), a kernel + memory-copy
# trace of the crate-shaped path inside a bench process, then the -m gpu suite
# and smoke.  Every GPU step has its own time limit; any failure stops the
# script (nothing retried).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r04}
export TMPDIR=/tmp
hostname > "$OUT/box_$TAG.txt"

if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python bench.py --profile-dir "$OUT/${TAG}_prof" \
      > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; tail -c 300 "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
fi

if [ "${COPYTRACE:-0}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
      -d "$PWD/$OUT/copytrace_$TAG" -o run -- python3 bench.py --steps 5 --warmup 2 --c5 off \
      --cpu-baseline off --pmc off --trace off --pcie off --c4 off \
      > "$OUT/copytrace_$TAG.json" 2> "$OUT/copytrace_$TAG.err"
  rc=$?; echo "copytrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi
