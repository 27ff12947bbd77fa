#!/bin/bash
# Round 4, VERDICT r3 item 4: codec streams per context (BFRS_CODEC_STREAMS:
# 0 = one per slot as in rounds 2-3, 4 / 8 = a fixed shared set) in the bench
# process (crate_api, after the device legs) and in a fresh process
# (tools/rayon_probe.py), alternated on one box; then a kernel trace of one
# bench process per mode (the runtime's blit-copy kernels per stream/queue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04e}
export TMPDIR=/tmp
COMMON="--steps 5 --warmup 2 --c5 off --cpu-baseline off --pmc off --trace off --pcie off --c4 off"
# modes: "<streams>:<copies>:<prefault>"; 0:slot:0 = rounds 2-3
for round in 1 2; do
  for mode in ${MODES:-0:slot:0 4:stream:0 4:stream:1 0:stream:1}; do
    IFS=: read ns cp pf <<< "$mode"
    BFRS_CODEC_STREAMS=$ns BFRS_CODEC_COPIES=$cp BFRS_PREFAULT_OUTPUTS=$pf timeout -k 10 300 python bench.py $COMMON \
        > "$OUT/sab_${TAG}_${ns}${cp}${pf}_$round.json" 2> "$OUT/sab_${TAG}_${ns}${cp}${pf}_$round.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench streams=$ns rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['crate_api']; print('bench mode', sys.argv[2], 'all_blocks', d['generate_parity_all_blocks_threads']['ms'], d['generate_parity_all_blocks_threads']['median_ms'], 'floor', d['generate_parity_all_blocks_threads']['floor_ms'], 'gp', d['generate_parity']['ms'], d['generate_parity']['median_ms'], 'touched', d['generate_parity']['touched_outputs_ms'], 'floor', d['link']['floor_generate_parity_ms'], 'rec', d['recover_segment_rs30_3']['ms'], 'child', (d.get('generate_parity_all_blocks_fresh_process') or {}).get('ms'))" "$OUT/sab_${TAG}_${ns}${cp}${pf}_$round.json" $mode
  done
done
for mode in ${TRACE_MODES:-}; do
  ns=${mode%%:*}; cp=${mode##*:}
  BFRS_CODEC_STREAMS=$ns BFRS_CODEC_COPIES=$cp timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$PWD/$OUT/sab_ct_${TAG}_$ns$cp" -o run -- python3 bench.py $COMMON \
      > "$OUT/sab_ct_${TAG}_$ns$cp.json" 2> "$OUT/sab_ct_${TAG}_$ns$cp.err"
  rc=$?; echo "trace mode=$mode rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
