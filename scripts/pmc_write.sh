#!/bin/bash
# PMC passes (counters only, no trace domains) over a short kbench of the
# store variants: write request sizes, write stalls, read request sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcw
mkdir -p $OUT
CMD="python3 tools/kbench.py --rounds 1 --iters 3 --variants ${VARS:-41,5,44}"
i=0
for set in "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_WR_UNCACHED_32B" \
           "TCC_EA0_WRREQ_STALL TCC_TOO_MANY_EA_WRREQS_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL" \
           "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM_CREDIT_STALL"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$PWD/$OUT/p$i" -o pmc -- $CMD \
      > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
