#!/bin/bash
# Round 6: archive soak on the final tree (the tier-3 commit's overlapped
# reservation changed after scripts/r06_soak.sh ran).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06soak2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/soak_archive.py --seconds 200 --readers 4 --seed $((0xA4C6)) \
    > $O/soak_archive.json 2> $O/soak_archive.err
rc=$?; echo "archive soak rc=$rc"; head -c 400 $O/soak_archive.json; echo
exit $rc
