#!/bin/bash
# Bench A/B of kernel variants on one box: VARIANTS="5 36" ROUNDS=2 bash scripts/gpu_ab_variant.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 "${ROUNDS:-2}"); do
  for v in $VARIANTS; do
    BFRS_KERNEL_VARIANT=$v timeout -k 10 200 python3 bench.py --cpu-baseline off --pcie off \
        --steps "${STEPS:-100}" > "gpurun_out/abv_${v}_$i.log" 2>&1 || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/abv_${v}_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('v$v', d['value'], r['launch_ms'], r['frac'], r['launch_ms_by_direction'])"
  done
done
