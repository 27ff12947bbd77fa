#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, no trace domains) of one
# gf_apply variant's launch loop (tools/pmc_kernel.py).
# usage: PMC_VARIANTS="58 73" TAG=x bash scripts/r02_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r02}
if [ "${LIST:-0}" = 1 ]; then
  timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/pmc_list_$TAG.txt" 2>&1; echo "list rc=$?"
fi
IFS=';' read -ra SETS <<< "${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES}"
i=0
for v in ${PMC_VARIANTS:-73}; do
  for set in "${SETS[@]}"; do
    i=$((i+1))
    BFRS_KERNEL_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv \
        -d "$PWD/$OUT/pmc_${TAG}_v${v}_$i" -o pmc -- python3 tools/pmc_kernel.py --n ${PMC_N:-10} \
        > "$OUT/pmc_${TAG}_v${v}_$i.log" 2>&1
    rc=$?; echo "v$v pass $i ($set) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
