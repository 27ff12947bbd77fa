#!/bin/bash
# BFRS_TRACE phase lines of crate_api's all-blocks figure: bench process vs
# the standalone probe (tools/rayon_probe.py), same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BFRS_TRACE=1 PROBE_MODES=pinned PROBE_REPS=2 timeout -k 10 200 python -u tools/rayon_probe.py \
    > gpurun_out/trace_probe.json 2> gpurun_out/trace_probe.err
rc=$?; echo "probe rc=$rc"; cat gpurun_out/trace_probe.json; [ $rc -eq 0 ] || exit $rc
BFRS_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --c5 off --cpu-baseline off \
    --pmc off --pcie off --c4 off > gpurun_out/trace_bench.json 2> gpurun_out/trace_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/trace_bench.json')); print(d['crate_api']['generate_parity_all_blocks_threads'])"
