#!/bin/bash
# Which part of the bench process slows crate_api's all-blocks figure?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 5 --warmup 2 --c5 off --cpu-baseline off --pmc off"
run() { name=$1; shift; timeout -k 10 300 $B "$@" > gpurun_out/crate_ab_$name.json 2> gpurun_out/crate_ab_$name.err; rc=$?
  echo "$name rc=$rc"; python -c "import json,sys; d=json.load(open('gpurun_out/crate_ab_$name.json')); c=d['crate_api']; print(c['generate_parity']['ms'], c['generate_parity_all_blocks_threads'])"; return $rc; }
run bare --pcie off --c4 off && run pcie --pcie auto --c4 off && run c4 --pcie off --c4 auto
