#!/bin/bash
# Round 4: host-batch pipeline depth (BFRS_PIPE_SLOTS: slab buffers and
# streams per context) against the PCIe-inclusive rate, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04z}
ARGS="--steps 5 --warmup 2 --c5 off --c4 off --cpu-baseline off --pmc off --trace off"
for v in ${VALS:-3 2 4 6 3}; do
  BFRS_PIPE_SLOTS=$v timeout -k 10 300 python bench.py $ARGS > "$OUT/pipes_${TAG}_$v.json" \
      2> "$OUT/pipes_${TAG}_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "slots=$v rc=$rc"; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))['pcie_inclusive']
print(sys.argv[2], d['encode_GiBps'], d['decode_GiBps'], d['encode_ms'], d['decode_ms'], d['decode_match'])" "$OUT/pipes_${TAG}_$v.json" $v
done
