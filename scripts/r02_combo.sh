#!/bin/bash
# kbench A/B (KB variants) then the whole GPU suite on the default build, then
# optionally the default bench line.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r02}
if [ -n "${KB:-}" ]; then
  bash scripts/r02_variants.sh || exit $?
fi
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; cut -c1-300 "$OUT/bench_$TAG.json"; exit $rc
fi
