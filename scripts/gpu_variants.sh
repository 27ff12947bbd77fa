#!/bin/bash
# Parity of every selectable codec variant (BFRS_KERNEL_VARIANT), then the full
# GPU suite on the default.  A crash (not a plain test failure) stops it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01}
for v in ${VARIANTS:-5 36 37 40 41 42}; do
  BFRS_KERNEL_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu \
      --timeout 240 --timeout-method thread -k "golden or mixed or random or multiphase or many" \
      > "$OUT/pytest_v${v}_$TAG.log" 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -1 "$OUT/pytest_v${v}_$TAG.log")"; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "default: $(tail -1 "$OUT/pytest_gpu_$TAG.log")"; exit $rc
