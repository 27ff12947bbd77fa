#!/bin/bash
# Config 5 read path: prefetch depth / workers A/B (bench.py --workload c5).
# CFGS: space-separated depth,workers pairs, run in the order given.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for cfg in ${CFGS:-4,2 8,2 16,2 16,4 32,4}; do
  d=${cfg%,*}; w=${cfg#*,}; i=$((i + 1))
  BFRS_PREFETCH_DEPTH=$d BFRS_PREFETCH_WORKERS=$w timeout -k 10 300 python bench.py --workload c5 \
      --cpu-baseline off > gpurun_out/c5pf_${i}_${d}_$w.json 2> gpurun_out/c5pf_${i}_${d}_$w.err
  rc=$?; echo "depth $d workers $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('gpurun_out/c5pf_${i}_${d}_$w.json')); print(d['value'], d['clean_read_MBps'], d['blake3_match'], d['stats_corrupted']['misses'])"
done
