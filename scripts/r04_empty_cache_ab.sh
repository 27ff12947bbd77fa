#!/bin/bash
# Round 4: torch's cached pinned host blocks given back before crate_api
# (BENCH_HOST_EMPTY_CACHE=1) or not, full bench runs alternating, one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04ec}
for v in 1 0 1 0; do
  BENCH_HOST_EMPTY_CACHE=$v timeout -k 10 300 python bench.py --pmc off --trace off --c5 off --cpu-baseline off \
      > "$OUT/ec_${TAG}_$v.json" 2> "$OUT/ec_${TAG}_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "empty=$v rc=$rc"; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))['crate_api']; a=d['generate_parity_all_blocks_threads']
print(sys.argv[2], a['ms'], a['median_ms'], a['floor_ms'], d['generate_parity']['ms'], d.get('pinned_host_before'))" "$OUT/ec_${TAG}_$v.json" $v
done
