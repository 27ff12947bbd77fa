#!/bin/bash
# c4_strong's golden check at N > 1 (stripes all-gathered, reassembled on rank
# 0), rehearsed with 2 and 4 ranks on one card over gloo at full C4 size.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --one-device --backend gloo --steps 3 --warmup 1 \
      --settle-ms 200 --pcie off > gpurun_out/c4_multirank_$n.json 2> gpurun_out/c4_multirank_$n.err
  rc=$?; echo "ranks $n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('gpurun_out/c4_multirank_$n.json')); p=d['parity_check']; print(d['n_gpus'], d['world_size_observed'], p['c4_encode'], p['c4_decode'], p['all_ok'])"
done
