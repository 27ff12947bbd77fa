#!/bin/bash
# Round-5 soaks on the final tree (GPU box).
#  1. A traced codec soak: rocprofv3 --kernel-trace (no --pmc) around
#     tools/soak.py, so that a fault names the dispatch that was running
#     (DESIGN.md §7c); the soak itself records what every thread had in
#     flight at its first failure (host copies included).  The traces are
#     kept only when the soak failed.  (--memory-copy-trace is not used: with
#     it rocprofv3 segfaults in __cxa_finalize at process exit and writes
#     nothing -- round 4's bench (r04a) and round 5's first traced soak
#     (r05s: 2,201 cases, 0 failures, then SIGSEGV at teardown).)
#  2. Plain soaks: codec (20% of cases at 8-40 MiB: the slab wrappers and
#     their fence), archive, BLAKE3.
# Each run has its own time limit; a failure stops here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r05}
SECS=${SECS:-150}
export TMPDIR=/tmp

if [ "${TRACED:-1}" = 1 ]; then
  mkdir -p "$OUT/soaktrace_$TAG"
  BFRS_PLAN_CACHE=16 BFRS_CODEC_SLOTS=2 timeout -k 10 300 \
      rocprofv3 --kernel-trace --output-format csv \
      -d "$PWD/$OUT/soaktrace_$TAG" -o soak -- \
      python3 tools/soak.py --seconds 60 --threads 6 --large --huge 0.2 --seed $((0x5B05)) \
      > "$OUT/soak_${TAG}_traced.json" 2> "$OUT/soak_${TAG}_traced.err"
  rc=$?; echo "traced codec soak rc=$rc"; tail -c 400 "$OUT/soak_${TAG}_traced.json"
  if [ $rc -eq 0 ]; then
    find "$OUT/soaktrace_$TAG" -name '*.csv' -size +1M -delete
  else
    exit $rc
  fi
fi

BFRS_PLAN_CACHE=16 BFRS_CODEC_SLOTS=2 timeout -k 10 $((SECS + 240)) \
    python3 tools/soak.py --seconds "$SECS" --threads 6 --large --huge 0.2 --seed $((0x5B15)) \
    > "$OUT/soak_${TAG}_codec.json" 2> "$OUT/soak_${TAG}_codec.err"
rc=$?; echo "codec soak rc=$rc"; tail -c 300 "$OUT/soak_${TAG}_codec.json"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 $((SECS + 240)) python3 tools/soak_archive.py --seconds "$SECS" --readers 4 \
    > "$OUT/soak_${TAG}_archive.json" 2> "$OUT/soak_${TAG}_archive.err"
rc=$?; echo "archive soak rc=$rc"; tail -c 300 "$OUT/soak_${TAG}_archive.json"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 $((SECS / 2 + 240)) python3 tools/soak_blake3.py --seconds $((SECS / 2)) \
    > "$OUT/soak_${TAG}_blake3.json" 2> "$OUT/soak_${TAG}_blake3.err"
rc=$?; echo "blake3 soak rc=$rc"; tail -c 300 "$OUT/soak_${TAG}_blake3.json"; [ $rc -eq 0 ] || exit $rc
echo "r05_soak done"
