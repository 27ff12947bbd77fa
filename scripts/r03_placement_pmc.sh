#!/bin/bash
# Round 3: what the slow placement mode is, with counters round 2 did not
# collect (GMI/IO read traffic and credit stalls, UTCL1 stall causes);
# one pass per counter group, each its own process, fast/slow copies compared
# WITHIN a pass (tools/placement_pmc.py).
# usage: TAG=x [PASSES="1 3"] bash scripts/r03_placement_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r03}
export TMPDIR=/tmp
SETS=("TCC_EA0_RDREQ_GMI_32B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_RDREQ_IO_32B_sum GRBM_GUI_ACTIVE"
      "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE"
      "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE")
for i in ${PASSES:-1 2 3}; do
  set=${SETS[$((i - 1))]}
  # a set over one pass's per-block limits makes rocprofv3 hang at start
  # (round 3's per-channel TCC pass): refuse it before the GPU is touched
  python3 tools/pmc_fit.py $set || exit 2
  timeout -s KILL 240 rocprofv3 --pmc $set --output-format csv -d "$PWD/$OUT/ppmc_${TAG}_$i" -o pmc \
      -- python3 tools/placement_pmc.py --copies ${COPIES:-6} --launches 20 > "$OUT/ppmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/placement_pmc.py --summarize "$OUT/ppmc_${TAG}_$i/pmc_counter_collection.csv" \
      --copies ${COPIES:-6} > "$OUT/ppmc_${TAG}_$i.json"
  rm -rf "$OUT/ppmc_${TAG}_$i"  # raw CSVs hold every torch fill kernel too (tens of MiB)
done
