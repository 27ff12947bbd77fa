#!/bin/bash
# Round 6: rehearsal of the driver's N = 8 launch on the one-GPU box with the
# final tree (torchrun, 8 ranks, every rank on cuda:0 over gloo, small sizes;
# 8 GPU processes, each behind its GPU-free supervisor).  Checks the launcher,
# supervisors, the all-gathers, c4_strong's stripes and c4_one_process with 8
# contexts, and the ordered teardown of every rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06r8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --one-device --backend gloo \
    --segments 8 --segment-bytes 1048576 --c4-segments 40 --steps 3 --warmup 1 --settle-ms 50 \
    > $O/line.json 2> $O/err.log
rc=$?; echo "torchrun 8 rc=$rc"; tail -c 1500 $O/line.json; echo; tail -5 $O/err.log
exit $rc
