set -u
mkdir -p gpurun_out
run() { name=$1; shift; env "$@" PROBE_MODES=pinned timeout -k 10 200 python -u tools/rayon_probe.py > gpurun_out/rayon_r03y_$name.json 2> gpurun_out/rayon_r03y_$name.err; rc=$?; echo "$name rc=$rc"; cat gpurun_out/rayon_r03y_$name.json; return $rc; }
run base X=1 && run torchsegs PROBE_TORCH_SEGS=1 && run pinned8 PROBE_PINNED_GIB=8 && run both PROBE_TORCH_SEGS=1 PROBE_PINNED_GIB=8
