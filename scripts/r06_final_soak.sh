#!/bin/bash
# Round 6, last product change (MADV_DONTFORK on the registered staging):
# the GPU suite, smoke, then a codec soak and an archive soak on that tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06fs
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
BFRS_PLAN_CACHE=16 timeout -k 10 300 python3 tools/soak.py --seconds 150 --threads 6 --large --huge 0.2 \
    --seed $((0x5C07)) --maps $O/codec.maps > $O/soak_codec.json 2> $O/soak_codec.err
rc=$?; echo "codec soak rc=$rc"; head -c 400 $O/soak_codec.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/soak_archive.py --seconds 120 --readers 4 --seed $((0xA4C7)) \
    > $O/soak_archive.json 2> $O/soak_archive.err
rc=$?; echo "archive soak rc=$rc"; head -c 400 $O/soak_archive.json; echo
exit $rc
