#!/bin/bash
# One kbench process per shard stagger (no layout switching inside a process).
# usage: VARIANTS=40 STAGGERS="12288 77824" TAG=x bash scripts/gpu_stagger_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for x in $STAGGERS; do
  for d in "" "--decode"; do
    timeout -k 10 120 python3 tools/kbench.py $d --variants "$VARIANTS" --stagger "$x" \
        --rounds "${ROUNDS:-5}" --iters 10 > "gpurun_out/kbs_${TAG}_${x}${d}.log" 2>&1 || exit $?
  done
done
