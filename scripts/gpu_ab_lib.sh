#!/bin/bash
# Bench A/B of two in-tree library builds on one box:
#   LIBS="libbfrs.so libbfrs_prev.so" ROUNDS=2 bash scripts/gpu_ab_lib.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 "${ROUNDS:-2}"); do
  for l in $LIBS; do
    BFRS_LIB=$l timeout -k 10 200 python3 bench.py --cpu-baseline off --pcie off \
        --steps "${STEPS:-100}" > "gpurun_out/abl_${l}_$i.log" 2>&1 || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/abl_${l}_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$l', d['value'], r['launch_ms'], r['frac'], r['launch_ms_by_direction'])"
  done
done
