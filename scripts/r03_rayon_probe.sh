#!/bin/bash
# The rayon-over-blocks shape of the crate path (tools/rayon_probe.py) under
# copy-thread caps and helper budgets ("-" = the library default); each run
# has its own time limit, any failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r03}
for t in ${THREADS:-8 4 2}; do
  for b in ${BUDGETS:--}; do
    [ "$b" = - ] && unset BFRS_HOST_COPY_BUDGET || export BFRS_HOST_COPY_BUDGET=$b
    f="$OUT/rayon_${TAG}_t${t}_b${b}"
    BFRS_HOST_COPY_THREADS=$t timeout -k 10 240 python -u tools/rayon_probe.py > "$f.json" 2> "$f.err"
    rc=$?; echo "threads $t budget $b rc=$rc"; cat "$f.json"; [ $rc -eq 0 ] || exit $rc
  done
done
if [ "${CRATE_PROBE:-0}" = 1 ]; then
  unset BFRS_HOST_COPY_BUDGET
  timeout -k 10 240 python -u tools/crate_probe.py > "$OUT/crate_probe_$TAG.json" 2> "$OUT/crate_probe_$TAG.err"
  rc=$?; echo "crate_probe rc=$rc"; cat "$OUT/crate_probe_$TAG.json"; [ $rc -eq 0 ] || exit $rc
fi
