#!/bin/bash
# Profiles the bench command: kernel trace + stats, then PMC passes for HBM
# traffic (FETCH_SIZE and WRITE_SIZE in separate passes; no trace domains
# combined with --pmc).  Outputs under gpurun_out/prof_$TAG*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
TAG=${TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
CMD="python3 bench.py --steps ${STEPS:-50} --warmup 30 --cpu-baseline off --pcie off"

timeout -k 10 600 python3 bench.py ${BENCH_EXTRA:-} > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench_$TAG.log"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$PWD/$OUT/prof_$TAG" -o run -- $CMD > "$OUT/prof_${TAG}.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 "$OUT/prof_${TAG}.log"; [ $rc -eq 0 ] || exit $rc

for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv \
      -d "$PWD/$OUT/prof_${TAG}_$c" -o pmc -- $CMD > "$OUT/prof_${TAG}_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; tail -1 "$OUT/prof_${TAG}_$c.log"; [ $rc -eq 0 ] || exit $rc
done
find "$OUT" -path "*prof_$TAG*" -name '*.csv' | head -20
