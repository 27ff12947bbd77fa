#!/bin/bash
# Round 6, second GPU call: the archive lifecycle tests (VERDICT r5 item 1,
# ADVICE r5), the pinning-rate probe with the registration forms (item 3),
# v76 vs the best LDS-DMA variant over eight placements (item 2), then the
# exit-time fault probes under the profiler flags of rounds 4-5 -- last,
# because a fault there ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06b
mkdir -p $O
export TMPDIR=/tmp
echo "tests"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_gpu_archive.py -k "closed_before or left_open or share_the_segment_pool or reconstructs or prefetch_settings or concurrent or tier2_handle" \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "pin probe"
timeout -k 10 180 python3 tools/pin_probe.py > $O/pin_probe.json 2> $O/pin_probe.err || { tail $O/pin_probe.err; exit 1; }
cat $O/pin_probe.json
echo "kernels over 8 placements"
for dir in enc dec; do
  flag=""; [ $dir = dec ] && flag="--decode"
  timeout -k 10 400 python3 tools/kbench.py $flag --variants 76,108 \
      --stagger 12288,16384,20480,28672,36864,45056,53248,61440 --rounds 3 --iters 10 \
      > $O/kb8_$dir.json 2> $O/kb8_$dir.err || { tail -20 $O/kb8_$dir.err; exit 1; }
  echo "$dir done"
done
echo "teardown: torch only under the r04/r05 profiler flags"
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d "$GRAFT_REPO_ROOT/$O/td_torch" -o td -- python3 "$GRAFT_REPO_ROOT/tools/teardown_probe.py" torch \
    --maps "$GRAFT_REPO_ROOT/$O/td_torch.maps" > "$GRAFT_REPO_ROOT/$O/td_torch.out" 2> "$GRAFT_REPO_ROOT/$O/td_torch.err"
rc=$?
echo "torch-only rc=$rc"
tail -5 "$GRAFT_REPO_ROOT/$O/td_torch.err"
[ $rc -eq 0 ] || exit 0
echo "teardown: bfrs under the same flags"
timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d "$GRAFT_REPO_ROOT/$O/td_bfrs" -o td -- python3 "$GRAFT_REPO_ROOT/tools/teardown_probe.py" bfrs \
    --maps "$GRAFT_REPO_ROOT/$O/td_bfrs.maps" > "$GRAFT_REPO_ROOT/$O/td_bfrs.out" 2> "$GRAFT_REPO_ROOT/$O/td_bfrs.err"
rc=$?
echo "bfrs rc=$rc"
tail -5 "$GRAFT_REPO_ROOT/$O/td_bfrs.err"
exit 0
