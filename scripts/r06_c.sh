#!/bin/bash
# Round 6, third GPU call: the GPU suite on the tree with huge-page registered
# staging buffers; a same-box A/B of the archive pipeline and of config 5
# (fresh and warm contexts) with hipHostMalloc (BFRS_PIN_MODE=malloc,
# measurement build) against registration; then the round-5 traced soak
# under rocprofv3 --memory-copy-trace (last: a fault there ends the call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06c
mkdir -p $O
export TMPDIR=/tmp
echo "gpu suite"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2; do
  for mode in malloc register; do
    echo "round $r $mode"
    BFRS_LIB=libbfrs_ab.so BFRS_PIN_MODE=$mode timeout -k 10 200 python3 tools/commit_bench.py \
        > $O/commit_${mode}_$r.json 2> $O/commit_${mode}_$r.err || { tail $O/commit_${mode}_$r.err; exit 1; }
    BFRS_LIB=libbfrs_ab.so BFRS_PIN_MODE=$mode timeout -k 10 200 python3 bench.py --workload c5 --no-supervisor \
        > $O/c5_${mode}_$r.json 2> $O/c5_${mode}_$r.err || { tail $O/c5_${mode}_$r.err; exit 1; }
  done
done
echo "traced soak"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d "$GRAFT_REPO_ROOT/$O/soaktrace" -o soak -- python3 "$GRAFT_REPO_ROOT/tools/soak.py" \
    --seconds 30 --threads 6 --large --huge 0.2 --seed $((0x5B06)) \
    --maps "$GRAFT_REPO_ROOT/$O/soak.maps" > "$GRAFT_REPO_ROOT/$O/soak_traced.json" 2> "$GRAFT_REPO_ROOT/$O/soak_traced.err"
rc=$?
echo "traced soak rc=$rc"
tail -3 "$GRAFT_REPO_ROOT/$O/soak_traced.err"
ls "$GRAFT_REPO_ROOT/$O/soaktrace" | head
exit 0
