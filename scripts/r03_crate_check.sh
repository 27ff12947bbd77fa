#!/bin/bash
# crate-shaped wrappers on one box: tools/crate_probe.py twice, then the bench's
# crate_api (other sub-objects off).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
for i in 1 2; do
  timeout -k 10 240 python -u tools/crate_probe.py > gpurun_out/crate_probe_${TAG}_$i.json 2> gpurun_out/crate_probe_${TAG}_$i.err
  rc=$?; echo "probe $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('gpurun_out/crate_probe_${TAG}_$i.json')); print({k: d[k] for k in d if k.startswith(('cabi_', 'recover_'))})"
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --c5 off --cpu-baseline off --pmc off --pcie off --c4 off \
    > gpurun_out/bench_crate_$TAG.json 2> gpurun_out/bench_crate_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/bench_crate_$TAG.json')); c=d['crate_api']; print(c['generate_parity'], c['recover_segment_rs30_3']['ms'], c['generate_parity_all_blocks_fresh_process']['ms'])"
