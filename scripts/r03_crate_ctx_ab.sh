#!/bin/bash
# crate_api's all-blocks figure on the bench's main context or on a new one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 5 --warmup 2 --c5 off --cpu-baseline off --pmc off --pcie off --c4 off"
for i in 1 2; do
  for c in new main; do
    BENCH_ALLBLOCKS_CTX=$c BENCH_ALLBLOCKS=first timeout -k 10 300 $B > gpurun_out/ctx_${c}_$i.json 2> gpurun_out/ctx_${c}_$i.err
    rc=$?; echo "$c $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python -c "import json; d=json.load(open('gpurun_out/ctx_${c}_$i.json')); c=d['crate_api']['generate_parity_all_blocks_threads']; print(c['ms'], c['median_ms'])"
  done
done
