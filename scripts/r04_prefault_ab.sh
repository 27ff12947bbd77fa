#!/bin/bash
# Round 4: fresh-output prefault variants, crate legs only, alternating in one
# box so host variance hits both.  MODE=populate: madvise(MADV_POPULATE_WRITE)
# (1, default) against one written byte per page (0).  MODE=early: the slab
# paths fault the outputs in from the start of the call (1) or after the last
# slab's copies (0); that knob was removed after r04n (worse).  MODE=parts:
# helper threads per fresh output, 4 against 1 (the encode default until r04v).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04m}
ARGS="--steps 5 --warmup 2 --c5 off --c4 off --pcie off --cpu-baseline off --pmc off --trace off"
MODE=${MODE:-populate}
case $MODE in
  populate) VAR=BFRS_PREFAULT_POPULATE; VALS="1 0 1 0";;
  early) VAR=BFRS_PREFAULT_EARLY; VALS="1 0 1 0";;
  parts) VAR=BFRS_PREFAULT_PARTS; VALS="4 1 4 1";;  # threads per output (r04v: encode 1 -> 4)
  huge) VAR=BFRS_PREFAULT_HUGE; VALS="1 0 1 0";;  # MADV_HUGEPAGE first (r04h2; knob removed)
esac
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python bench.py $ARGS > "$OUT/pf_${TAG}_${MODE}$v.json" 2> "$OUT/pf_${TAG}_${MODE}$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "$VAR=$v rc=$rc"; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))['crate_api']; g=d['generate_parity']; r=d['recover_segment_rs30_3']
a=d['generate_parity_all_blocks_threads']; f=d.get('generate_parity_all_blocks_fresh_process',{})
print(sys.argv[2], a['ms'], g['ms'], g['touched_outputs_ms'], r['ms'], r['touched_output_ms'], f.get('ms'))" "$OUT/pf_${TAG}_${MODE}$v.json" $v
done
