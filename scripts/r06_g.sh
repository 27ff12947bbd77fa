#!/bin/bash
# Round 6: the tier-3 commit reserving its second block buffer and parity
# slots beside block 0's fill; the archive GPU tests and the pipeline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_archive.py \
    > $O/archive_tests.log 2>&1 || { tail -30 $O/archive_tests.log; exit 1; }
tail -1 $O/archive_tests.log
for r in 1 2; do
  timeout -k 10 200 python3 tools/commit_bench.py > $O/commit_$r.json 2> $O/commit_$r.err || { tail $O/commit_$r.err; exit 1; }
  head -c 400 $O/commit_$r.json; echo
done
timeout -k 10 300 python3 bench.py --workload c5 --no-supervisor > $O/c5.json 2> $O/c5.err || { tail $O/c5.err; exit 1; }
tail -c 600 $O/c5.json
