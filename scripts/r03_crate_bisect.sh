#!/bin/bash
# crate_api's all-blocks figure in bench processes that do less before it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --c5 off --cpu-baseline off --pmc off --pcie off --c4 off"
run() { name=$1; shift; timeout -k 10 300 $B "$@" > gpurun_out/bisect_$name.json 2> gpurun_out/bisect_$name.err; rc=$?
  echo "$name rc=$rc"; [ $rc -eq 0 ] || return $rc
  python -c "import json; d=json.load(open('gpurun_out/bisect_$name.json')); c=d['crate_api']['generate_parity_all_blocks_threads']; print(c['ms'], c['median_ms'])"; }
run minimal --steps 1 --warmup 0 --settle-ms 0 && run default --steps 5 --warmup 2 && run minimal2 --steps 1 --warmup 0 --settle-ms 0
