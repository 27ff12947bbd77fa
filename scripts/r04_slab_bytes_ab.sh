#!/bin/bash
# Round 4: host-batch slab width (BFRS_SLAB_BYTES) against the PCIe-inclusive
# rate (bench pcie_inclusive: C2 from pinned host buffers), one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04y}
ARGS="--steps 5 --warmup 2 --c5 off --c4 off --cpu-baseline off --pmc off --trace off"
for v in 8 4 16 32 8; do
  BFRS_SLAB_BYTES=$((v << 20)) timeout -k 10 300 python bench.py $ARGS > "$OUT/slabb_${TAG}_$v.json" \
      2> "$OUT/slabb_${TAG}_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "slab=$v rc=$rc"; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))['pcie_inclusive']
print(sys.argv[2], d['encode_GiBps'], d['decode_GiBps'], d['encode_ms'], d['decode_ms'], d['decode_match'])" "$OUT/slabb_${TAG}_$v.json" $v
done
