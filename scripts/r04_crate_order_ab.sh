#!/bin/bash
# Round 4: the crate_api leg before / after pcie_inclusive in full default
# bench runs (BENCH_CRATE_FIRST=1 / unset), alternating, one box (r04co: no
# effect; the knob was removed from bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04co}
for v in 1 0 1 0; do
  BENCH_CRATE_FIRST=$v timeout -k 10 300 python bench.py --pmc off --trace off --c5 off --cpu-baseline off \
      > "$OUT/co_${TAG}_$v.json" 2> "$OUT/co_${TAG}_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "first=$v rc=$rc"; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))['crate_api']; a=d['generate_parity_all_blocks_threads']
print(sys.argv[2], a['ms'], a['median_ms'], a['floor_ms'], d['generate_parity']['ms'], d['recover_segment_rs30_3']['ms'])" "$OUT/co_${TAG}_$v.json" $v
done
