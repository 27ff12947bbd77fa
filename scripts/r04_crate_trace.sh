#!/bin/bash
# Round 4, VERDICT r3 item 4: kernel traces (queue / stream of every dispatch,
# the runtime's blit-copy kernels included) of C2's five blocks on five
# threads -- once in a fresh process (tools/rayon_probe.py), once inside a
# bench process after its device work (crate_api leg).  No --pmc, no
# memory-copy domain (that pass crashed at exit in r04a).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04c}
export TMPDIR=/tmp
PROBE_MODES=pinned PROBE_REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$PWD/$OUT/ct_probe_$TAG" -o run -- python3 tools/rayon_probe.py \
    > "$OUT/ct_probe_$TAG.json" 2> "$OUT/ct_probe_$TAG.err"
rc=$?; echo "probe rc=$rc"; tail -c 400 "$OUT/ct_probe_$TAG.json"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$PWD/$OUT/ct_bench_$TAG" -o run -- python3 bench.py --steps 5 --warmup 2 --c5 off \
    --cpu-baseline off --pmc off --trace off --pcie off --c4 off \
    > "$OUT/ct_bench_$TAG.json" 2> "$OUT/ct_bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
