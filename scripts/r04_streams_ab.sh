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
for round in 1 2; do
  for ns in 0 4 8; do
    BFRS_CODEC_STREAMS=$ns timeout -k 10 300 python bench.py $COMMON > "$OUT/sab_${TAG}_${ns}_$round.json" \
        2> "$OUT/sab_${TAG}_${ns}_$round.err"
    rc=$?; [ $rc -eq 0 ] || { echo "bench streams=$ns rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['crate_api']; print('bench streams', sys.argv[2], 'all_blocks', d['generate_parity_all_blocks_threads']['ms'], d['generate_parity_all_blocks_threads']['median_ms'], 'floor', d['generate_parity_all_blocks_threads']['floor_ms'], 'gp', d['generate_parity']['ms'], 'rec', d['recover_segment_rs30_3']['ms'], 'child', (d.get('generate_parity_all_blocks_fresh_process') or {}).get('ms'))" "$OUT/sab_${TAG}_${ns}_$round.json" $ns
  done
done
for ns in 0 4; do
  BFRS_CODEC_STREAMS=$ns timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$PWD/$OUT/sab_ct_${TAG}_$ns" -o run -- python3 bench.py $COMMON \
      > "$OUT/sab_ct_${TAG}_$ns.json" 2> "$OUT/sab_ct_${TAG}_$ns.err"
  rc=$?; echo "trace streams=$ns rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
