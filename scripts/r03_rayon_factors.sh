#!/bin/bash
# Which process state slows the rayon shape (tools/rayon_probe.py variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
run() { name=$1; shift; env "$@" PROBE_MODES=pinned timeout -k 10 200 python -u tools/rayon_probe.py > gpurun_out/rayon_${TAG}_$name.json 2> gpurun_out/rayon_${TAG}_$name.err; rc=$?; echo "$name rc=$rc"; cat gpurun_out/rayon_${TAG}_$name.json; return $rc; }
for v in ${VARIANTS:-base}; do
  case $v in
    base) run base X=1 ;;
    torchsegs) run torchsegs PROBE_TORCH_SEGS=1 ;;
    pinned8) run pinned8 PROBE_PINNED_GIB=8 ;;
    gpuwork) run gpuwork PROBE_GPU_WORK=10 ;;
    gpuwork_keep) run gpuwork_keep PROBE_GPU_WORK=10 PROBE_KEEP_HBM=1 ;;
  esac || exit 1
done
