#!/bin/bash
# rocprofv3 of the driver's exact bench command (round 3): kernel trace + stats, then
# PMC passes FETCH_SIZE and WRITE_SIZE (separate runs, no trace domains with
# --pmc).  Outputs under gpurun_out/prof_$TAG*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r03}
export TMPDIR=/tmp
hostname > "$OUT/prof_${TAG}_box.txt"
CMD="python3 bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$PWD/$OUT/prof_$TAG" -o run -- $CMD > "$OUT/prof_${TAG}.log" 2>&1
rc=$?; echo "trace rc=$rc"; tail -c 400 "$OUT/prof_${TAG}.log"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 900 rocprofv3 --pmc $c --output-format csv \
      -d "$PWD/$OUT/prof_${TAG}_$c" -o pmc -- $CMD > "$OUT/prof_${TAG}_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
