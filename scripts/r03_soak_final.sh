#!/bin/bash
# Final-tree soaks (round 3): codec soak with multi-MiB and 8-40 MiB shards
# over the pinned staging (threaded copies under the shared budget), then the
# archive soak (commit pipelines, repair, concurrent readers).  Each run has
# its own time limit; a failure stops here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
SECS=${SECS:-180}
BFRS_PLAN_CACHE=16 BFRS_CODEC_SLOTS=2 timeout -k 10 $((SECS + 180)) \
    python tools/soak.py --seconds "$SECS" --threads 6 --large --huge 0.05 --seed $((0x5B00)) \
    > "$OUT/soak_r03_final_codec.json" 2> "$OUT/soak_r03_final_codec.err"
rc=$?; echo "codec rc=$rc"; tail -c 600 "$OUT/soak_r03_final_codec.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 $((SECS + 180)) python tools/soak_archive.py --seconds "$SECS" --seed $((0xA5C3)) \
    > "$OUT/soak_r03_final_archive.json" 2> "$OUT/soak_r03_final_archive.err"
rc=$?; echo "archive rc=$rc"; tail -c 600 "$OUT/soak_r03_final_archive.json"; exit $rc
