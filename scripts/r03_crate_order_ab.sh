#!/bin/bash
# crate_api's all-blocks figure timed first (right after the link settle) or
# after the single-block figures; alternating runs, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 5 --warmup 2 --c5 off --cpu-baseline off --pmc off --pcie off --c4 off"
for i in 1 2; do
  for o in first late; do
    BENCH_ALLBLOCKS=$o timeout -k 10 300 $B > gpurun_out/order_${o}_$i.json 2> gpurun_out/order_${o}_$i.err
    rc=$?; echo "$o $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.load(open('gpurun_out/order_${o}_$i.json')); c=d['crate_api']; print(c['generate_parity']['ms'], c['recover_segment_rs30_3']['ms'], c['generate_parity_all_blocks_threads']['ms'], c['generate_parity_all_blocks_threads']['median_ms'])"
  done
done
