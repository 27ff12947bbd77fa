#!/bin/bash
# Phased-kernel session: parity of the phased variants, then an interleaved
# kbench (encode and decode) against the default ring kernel.  A crash stops
# the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01w}
stop_if_crash() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: $2 exited $1"; exit "$1"; fi; }
for v in ${VARIANTS_PARITY:-24 25 26}; do
  BFRS_KERNEL_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu \
      --timeout 120 --timeout-method thread > "$OUT/pytest_v${v}_$TAG.log" 2>&1
  rc=$?; echo "variant $v parity rc=$rc"; tail -2 "$OUT/pytest_v${v}_$TAG.log"; stop_if_crash $rc "parity v$v"
  [ $rc -ne 0 ] && exit 1
done
for d in "" "--decode"; do
  timeout -k 10 300 python -u tools/kbench.py --rounds 4 --iters 30 $d --variants ${KB_VARIANTS:-5,24,25,26,21,22,9} \
      > "$OUT/kbench${d}_$TAG.log" 2>&1
  rc=$?; echo "kbench $d rc=$rc"; grep -E '"v' "$OUT/kbench${d}_$TAG.log" | head -30; stop_if_crash $rc kbench
done
