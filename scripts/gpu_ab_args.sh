#!/bin/bash
# Bench A/B of bench.py argument sets on one box:
#   A="--layout single" B="--layout separate" ROUNDS=2 bash scripts/gpu_ab_args.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in $(seq 1 "${ROUNDS:-2}"); do
  for k in A B; do
    timeout -k 10 200 python3 bench.py --cpu-baseline off --pcie off --steps "${STEPS:-100}" ${!k} \
        > "gpurun_out/aba_${k}_$i.log" 2>&1 || exit $?
    python3 -c "import json;d=json.loads(open('gpurun_out/aba_${k}_$i.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$k', d['value'], r['launch_ms'], r['frac'], r['launch_ms_by_direction'])"
  done
done
