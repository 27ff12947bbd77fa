#!/bin/bash
# A/B of kernel variants in one process per direction (tools/kbench.py).
# usage: VARIANTS=5,36 STAGGER=12288 TAG=x bash scripts/gpu_kb.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python3 tools/kbench.py --variants "$VARIANTS" --stagger "${STAGGER:-12288}" \
    --rounds "${ROUNDS:-3}" --iters 10 > "gpurun_out/kb_${TAG}_enc.log" 2>&1 || exit $?
timeout -k 10 240 python3 tools/kbench.py --decode --variants "$VARIANTS" --stagger "${STAGGER:-12288}" \
    --rounds "${ROUNDS:-3}" --iters 10 > "gpurun_out/kb_${TAG}_dec.log" 2>&1
