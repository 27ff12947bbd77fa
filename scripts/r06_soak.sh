#!/bin/bash
# Round 6 soaks on the changed code paths only: the codec
# (slots on huge-page registered memory) and the archive pipeline (pre-pinning
# at open, one reconstruction arena per context, pool cap, detach).  No
# profiler: --memory-copy-trace corrupts host-batch copies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06soak
mkdir -p $O
export TMPDIR=/tmp
BFRS_PLAN_CACHE=16 timeout -k 10 400 python3 tools/soak.py --seconds 300 --threads 6 --large --huge 0.2 \
    --seed $((0x5C06)) --maps $O/codec.maps > $O/soak_codec.json 2> $O/soak_codec.err
rc=$?; echo "codec soak rc=$rc"; head -c 400 $O/soak_codec.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/soak_archive.py --seconds 200 --readers 4 > $O/soak_archive.json 2> $O/soak_archive.err
rc=$?; echo "archive soak rc=$rc"; head -c 400 $O/soak_archive.json; echo
exit $rc
