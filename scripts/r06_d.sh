#!/bin/bash
# Round 6, fourth GPU call.  The traced soak of call 3 (rocprofv3
# --kernel-trace --memory-copy-trace) reported 13 host-batch mismatches and
# ~1,000 "bad original signal value in async_copy_handler" lines from the
# profiler: is that the tracer or the tree?
#   1. the same soak, no profiler, this tree (60 s)
#   2. config 5 and the archive pipeline with the open-time pre-pinning
#   3. the soak under --kernel-trace only, this tree
#   4. the soak under --kernel-trace --memory-copy-trace with round 5's
#      library (libbfrs_r05.so, built from d893ca0), last: the profiler's
#      exit-time fault ends the call
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
echo "plain soak"
timeout -k 10 150 python3 tools/soak.py --seconds 60 --threads 6 --large --huge 0.2 --seed $((0x5B06)) \
    --maps $O/soak_plain.maps > $O/soak_plain.json 2> $O/soak_plain.err
echo "plain soak rc=$?"; head -c 300 $O/soak_plain.json; echo
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --workload c5 --no-supervisor > $O/c5_$r.json 2> $O/c5_$r.err || { tail $O/c5_$r.err; exit 1; }
done
timeout -k 10 200 python3 tools/commit_bench.py > $O/commit.json 2> $O/commit.err || { tail $O/commit.err; exit 1; }
echo "kernel-trace soak"
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d "$R/$O/kt" -o soak -- \
    python3 "$R/tools/soak.py" --seconds 30 --threads 6 --large --huge 0.2 --seed $((0x5B06)) \
    > "$R/$O/soak_kt.json" 2> "$R/$O/soak_kt.err"
rc=$?; echo "kernel-trace soak rc=$rc"; head -c 300 "$R/$O/soak_kt.json"; echo
[ $rc -eq 0 ] || exit 0
echo "memcopy-trace soak, round-5 library"
BFRS_LIB=libbfrs_r05.so timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d "$R/$O/mct" -o soak -- python3 "$R/tools/soak.py" --seconds 30 --threads 6 --large --huge 0.2 \
    --seed $((0x5B06)) --maps "$R/$O/soak_mct_r05.maps" > "$R/$O/soak_mct_r05.json" 2> "$R/$O/soak_mct_r05.err"
echo "memcopy-trace soak (r05 lib) rc=$?"; head -c 300 "$R/$O/soak_mct_r05.json"; echo
exit 0
