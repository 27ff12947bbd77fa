#!/bin/bash
# The rayon-over-blocks shape of the crate path (tools/rayon_probe.py) under
# copy-thread caps; each run has its own time limit, any failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r03}
for t in ${THREADS:-8 4 2}; do
  BFRS_HOST_COPY_THREADS=$t timeout -k 10 240 python -u tools/rayon_probe.py \
      > "$OUT/rayon_${TAG}_t$t.json" 2> "$OUT/rayon_${TAG}_t$t.err"
  rc=$?; echo "threads $t rc=$rc"; cat "$OUT/rayon_${TAG}_t$t.json"; [ $rc -eq 0 ] || exit $rc
done
