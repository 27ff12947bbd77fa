#!/bin/bash
# Round 4, VERDICT r3 item 4: is the slow crate path inside the bench process
# caused by the pinned host memory the earlier legs leave in torch's caching
# host allocator (c4_strong + pcie_inclusive: ~17 GB)?  Same box, three bench
# processes: legs before crate_api on / off / on + torch host cache emptied.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04d}
COMMON="--steps 5 --warmup 2 --c5 off --cpu-baseline off --pmc off --trace off"
for v in on off on_empty on; do
  case $v in
    on) args="$COMMON"; env="";;
    off) args="$COMMON --pcie off --c4 off"; env="";;
    on_empty) args="$COMMON"; env="BENCH_HOST_EMPTY_CACHE=1";;
  esac
  env $env BFRS_TRACE=1 timeout -k 10 300 python bench.py $args > "$OUT/crate_ab_${TAG}_$v.json" \
      2> "$OUT/crate_ab_${TAG}_$v.err"
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['crate_api']; print(sys.argv[2], d['generate_parity_all_blocks_threads']['ms'], d['generate_parity_all_blocks_threads']['median_ms'], d['generate_parity']['ms'], d['recover_segment_rs30_3']['ms'], d.get('pinned_host_before'))" "$OUT/crate_ab_${TAG}_$v.json" $v
done
