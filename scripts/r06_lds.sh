#!/bin/bash
# Round 6, VERDICT r5 item 2: the LDS-DMA input ring (v107-v109, measurement
# build) -- parity first, then the traffic probe and the kernels over several
# HBM placements, v76 beside them in the same process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_lds
mkdir -p $O
echo "parity"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread \
    tests/test_gpu_parity.py -k lds_dma_variants > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
echo "traffic probe"
timeout -k 10 240 ./tools/membench8 ldsplace > $O/mb8_ldsplace.jsonl 2>&1 || exit $?
echo "kernels"
for dir in enc dec; do
  flag=""; [ $dir = dec ] && flag="--decode"
  timeout -k 10 300 python3 tools/kbench.py $flag --variants "${VARIANTS:-76,107,108,109}" \
      --stagger "${STAGGER:-12288,16384,20480,28672}" --rounds "${ROUNDS:-3}" --iters 10 \
      > $O/kb_$dir.json 2> $O/kb_$dir.err || { tail -20 $O/kb_$dir.err; exit 1; }
  echo "$dir done"
done
