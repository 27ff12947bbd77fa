#!/bin/bash
# Round-3 codec soaks (tools/soak.py) over both codec-object stagings and idle-slot
# counts, wrappers included.  Each run has its own time limit; a failure stops here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
SECS=${SECS:-90}
for cfg in "pinned 2" "direct 0" "pinned 0"; do
  set -- $cfg
  tag="soak_r03_${1}_slots$2"
  BFRS_PLAN_CACHE=16 BFRS_CODEC_STAGING=$1 BFRS_CODEC_SLOTS=$2 timeout -k 10 $((SECS + 120)) \
      python tools/soak.py --seconds "$SECS" --threads 6 --large --seed $((0x5A00 + $2)) \
      > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  rc=$?; echo "$tag rc=$rc"; tail -c 400 "$OUT/$tag.json"; [ $rc -eq 0 ] || exit $rc
done
