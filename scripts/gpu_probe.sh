#!/bin/bash
# Kernel A/B session: full GPU tests, parity of the experimental variants,
# interleaved kbench of the variants, membench2 pattern probes (last: a
# measurement tool, not product code).  A crash stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
TAG=${TAG:-r01k}
stop_if_crash() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "STOP: $2 exited $1"; exit "$1"; fi; }

timeout -k 10 600 python -m pytest tests -q -m gpu -rf > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu_$TAG.log"; stop_if_crash $rc pytest
for v in ${VARIANTS_PARITY:-10 11 12}; do
  BFRS_KERNEL_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu \
      -k "golden or mixed or random or multiphase" > "$OUT/pytest_v${v}_$TAG.log" 2>&1
  rc=$?; echo "variant $v parity rc=$rc"; tail -1 "$OUT/pytest_v${v}_$TAG.log"; stop_if_crash $rc "parity v$v"
done
timeout -k 10 400 python tools/kbench.py --rounds 4 --iters 30 --variants ${KB_VARIANTS:-5,10,11,12,9} \
    > "$OUT/kbench_$TAG.log" 2>&1
rc=$?; echo "kbench rc=$rc"; grep -E '"v|"ms"|GBps' "$OUT/kbench_$TAG.log" | head -30; stop_if_crash $rc kbench
if [ "${MEMBENCH:-1}" = 1 ]; then
  timeout -k 10 300 ./tools/membench2 > "$OUT/membench2_$TAG.log" 2> "$OUT/membench2_${TAG}.err"
  rc=$?; echo "membench2 rc=$rc"; cat "$OUT/membench2_$TAG.log"; tail -2 "$OUT/membench2_${TAG}.err"
fi
