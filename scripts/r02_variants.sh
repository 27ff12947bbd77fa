#!/bin/bash
# Parity of candidate kernel variants (full test_gpu_parity.py each), then a
# same-process A/B (tools/kbench.py) and optional membench8 probe sets.
# usage: VARIANTS="70 71" KB=58,70,71,72 MB_SET=occ TAG=x bash scripts/r02_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r02}
for v in ${VARIANTS:-}; do
  BFRS_KERNEL_VARIANT=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
      --timeout 240 --timeout-method thread > "$OUT/pytest_v${v}_$TAG.log" 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -1 "$OUT/pytest_v${v}_$TAG.log")"; [ $rc -eq 0 ] || exit $rc
done
if [ -n "${KB:-}" ]; then
  timeout -k 10 300 python3 tools/kbench.py --variants "$KB" --stagger "${STAGGER:-12288}" --rounds "${ROUNDS:-3}" --tpw "${TPW:-0}" \
      --iters 10 > "$OUT/kb_${TAG}_enc.log" 2>&1
  rc=$?; echo "kbench enc rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 tools/kbench.py --decode --variants "$KB" --stagger "${STAGGER:-12288}" \
      --rounds "${ROUNDS:-3}" --tpw "${TPW:-0}" --segments "${SEGS:-128}" --iters 10 > "$OUT/kb_${TAG}_dec.log" 2>&1
  rc=$?; echo "kbench dec rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${MB_SET:-}" ]; then
  timeout -k 10 300 ./tools/membench8 "$MB_SET" > "$OUT/mb8_$TAG.jsonl" 2>&1
  rc=$?; echo "membench8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH_VARIANT:-}" ]; then
  BFRS_KERNEL_VARIANT=$BENCH_VARIANT timeout -k 10 300 python bench.py --cpu-baseline off --pcie off \
      > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
  rc=$?; echo "bench rc=$rc"; cut -c1-400 "$OUT/bench_$TAG.json"; exit $rc
fi
