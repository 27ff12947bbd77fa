#!/bin/bash
# Round-3 GPU-box session: the -m gpu suite, smoke, the driver's bench command,
# and a rocprofv3 kernel trace of that same command.  Every GPU step has its
# own time limit; any failure stops the script (nothing retried).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r03}
BENCH_CMD=${BENCH_CMD:-"bench.py --gpus 1 --steps 20 --warmup 5"}

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
      ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc

  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi

if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python $BENCH_CMD > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; tail -c 600 "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
fi

if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$OUT/prof_$TAG" -o run -- python3 $BENCH_CMD \
      > "$OUT/prof_$TAG.json" 2> "$OUT/prof_$TAG.err"
  rc=$?; echo "rocprof rc=$rc"; tail -c 300 "$OUT/prof_$TAG.json"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/prof_$TAG" -name '*stats*'
fi
