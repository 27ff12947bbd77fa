#!/bin/bash
# Round-2 first GPU session: GPU parity suite, HBM probes (tools/membench8),
# default bench.  Each GPU step has its own time limit; stop on any failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r02a}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./tools/membench8 ${MB_SET:-all} > "$OUT/mb8_$TAG.jsonl" 2>&1
rc=$?; echo "membench8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cut -c1-600 "$OUT/bench_$TAG.json"; exit $rc
