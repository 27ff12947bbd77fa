#!/bin/bash
# Round-4 final-tree soaks: the codec soak with 8-40 MiB shards at 20% (the
# slab-pipelined generate_parity / recover_segment_rs30_3 wrappers, RS(30,3)
# recovers at 16-20 MiB shards), then the archive soak and the BLAKE3 soak.
# (r04s/r04fs also registered the inputs of 30% of the multi-MiB wrapper cases;
# r04fs faulted the GPU and host registration was removed)
# Each run has its own time limit; a failure stops here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
SECS=${SECS:-150}
TAG=${TAG:-r04}
BFRS_PLAN_CACHE=16 BFRS_CODEC_SLOTS=2 timeout -k 10 $((SECS + 240)) \
    python tools/soak.py --seconds "$SECS" --threads 6 --large --huge 0.2 --seed $((0x5B04)) \
    > "$OUT/soak_${TAG}_codec.json" 2> "$OUT/soak_${TAG}_codec.err"
rc=$?; echo "codec rc=$rc"; tail -c 700 "$OUT/soak_${TAG}_codec.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 $((SECS + 180)) python tools/soak_archive.py --seconds "$SECS" --seed $((0xA5C4)) \
    > "$OUT/soak_${TAG}_archive.json" 2> "$OUT/soak_${TAG}_archive.err"
rc=$?; echo "archive rc=$rc"; tail -c 400 "$OUT/soak_${TAG}_archive.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 $((SECS + 120)) python tools/soak_blake3.py --seconds "$SECS" \
    > "$OUT/soak_${TAG}_blake3.json" 2> "$OUT/soak_${TAG}_blake3.err"
rc=$?; echo "blake3 rc=$rc"; tail -c 400 "$OUT/soak_${TAG}_blake3.json"; exit $rc
