#!/bin/bash
# Round 6, crate path A/B: the codec slots on huge-page registered memory
# (default) against hipHostMalloc (BFRS_PIN_MODE=malloc, measurement build),
# alternating, then the driver argv once (the probe passes' script path fix).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06f
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for mode in malloc register; do
    echo "round $r $mode"
    BFRS_LIB=libbfrs_ab.so BFRS_PIN_MODE=$mode timeout -k 10 120 python3 tools/crate_probe.py \
        > $O/crate_${mode}_$r.json 2> $O/crate_${mode}_$r.err || { tail $O/crate_${mode}_$r.err; exit 1; }
    BFRS_LIB=libbfrs_ab.so BFRS_PIN_MODE=$mode timeout -k 10 120 python3 tools/rayon_probe.py \
        > $O/rayon_${mode}_$r.json 2> $O/rayon_${mode}_$r.err || { tail $O/rayon_${mode}_$r.err; exit 1; }
  done
done
echo "driver argv"
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 $O/bench.err
exit $rc
