#!/bin/bash
# Rehearsal of the driver's N = 8 launch on one card: torchrun, 8 ranks, all on
# device 0 over gloo, small sizes (the real SCALE run is the driver's).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --one-device --backend gloo \
    --segments 8 --segment-bytes 1048576 --c4-segments 40 --steps 2 --warmup 1 --settle-ms 20 \
    > gpurun_out/torchrun8_r03.json 2> gpurun_out/torchrun8_r03.err
rc=$?; echo "torchrun rc=$rc"; grep -a '^{"metric"' gpurun_out/torchrun8_r03.json | head -c 900; exit $rc
