#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash (not a plain test failure)
# stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}

stop_if_crash() {  # $1 = rc, $2 = step
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then
    echo "STOP: $2 exited $1"; exit "$1"
  fi
}

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu -rf > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu_$TAG.log"; stop_if_crash $rc pytest

  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"; stop_if_crash $rc smoke
fi

if [ "${READPATH:-0}" = 1 ]; then
  timeout -k 10 900 python bench.py --workload c5 ${READPATH_ARGS:-} > "$OUT/readpath_$TAG.log" 2>&1
  rc=$?; echo "readpath rc=$rc"; tail -3 "$OUT/readpath_$TAG.log"; stop_if_crash $rc readpath
fi

timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench_$TAG.log"; [ $rc -eq 0 ] || exit $rc

if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$OUT/prof_$TAG" -o run -- python bench.py --steps 10 --warmup 3 --cpu-baseline off \
      > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof_$TAG.log"; [ $rc -eq 0 ] || exit $rc
  find "$OUT/prof_$TAG" -name '*stats*' | head
fi
