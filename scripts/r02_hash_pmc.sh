#!/bin/bash
# Device BLAKE3 (tools/hash_bench.py): kernel trace + one PMC pass (clock,
# VALU busy) to back DESIGN.md §7b's "VALU-bound".  Outputs gpurun_out/hash_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 300 python3 tools/hash_bench.py > "$OUT/hash_$TAG.json" 2>&1
rc=$?; echo "hash_bench rc=$rc"; tail -2 "$OUT/hash_$TAG.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/hash_trace_$TAG" -o run \
    -- python3 tools/hash_bench.py > "$OUT/hash_trace_$TAG.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv \
    -d "$PWD/$OUT/hash_pmc_$TAG" -o pmc -- python3 tools/hash_bench.py > "$OUT/hash_pmc_$TAG.log" 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
