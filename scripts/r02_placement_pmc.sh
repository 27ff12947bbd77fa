#!/bin/bash
# Placement study under PMC (tools/placement_pmc.py): one pass per counter
# group, each its own process, so fast/slow copies are compared WITHIN a pass.
# usage: TAG=x [PASSES="1 3"] bash scripts/r02_placement_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r02}
export TMPDIR=/tmp
SETS=("TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_PENDING_STALL_CYCLES_sum"
      "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE"
      "SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
for i in ${PASSES:-1 2 3}; do
  set=${SETS[$((i - 1))]}
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$PWD/$OUT/ppmc_${TAG}_$i" -o pmc \
      -- python3 tools/placement_pmc.py --copies ${COPIES:-6} --launches 20 > "$OUT/ppmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/placement_pmc.py --summarize "$OUT/ppmc_${TAG}_$i/pmc_counter_collection.csv" \
      --copies ${COPIES:-6} > "$OUT/ppmc_${TAG}_$i.json"
  rm -rf "$OUT/ppmc_${TAG}_$i"  # raw CSVs hold every torch fill kernel too (tens of MiB)
done
