#!/bin/bash
# Round 4: C2's five blocks on five threads in a fresh process
# (tools/rayon_probe.py) per copy mode -- pinned staging / registered inputs,
# copies on each object's stream (slot) / through the context's FIFO copy
# streams (stream) -- with a kernel trace of each (the runtime's blit-copy
# kernels per stream and queue), then the bench process's crate_api per mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p "$OUT"
TAG=${TAG:-r04i}
export TMPDIR=/tmp
for cp in slot stream; do
  BFRS_CODEC_COPIES=$cp PROBE_MODES=pinned,pinned_reg PROBE_REPS=4 timeout -k 10 240 rocprofv3 \
      --kernel-trace --stats --output-format csv -d "$PWD/$OUT/reg_${TAG}_$cp" -o run -- \
      python3 tools/rayon_probe.py > "$OUT/reg_${TAG}_$cp.json" 2> "$OUT/reg_${TAG}_$cp.err"
  rc=$?; echo "probe copies=$cp rc=$rc"; tail -c 600 "$OUT/reg_${TAG}_$cp.json"; [ $rc -eq 0 ] || exit $rc
done
COMMON="--steps 5 --warmup 2 --c5 off --cpu-baseline off --pmc off --trace off --pcie off --c4 off"
for cp in slot stream; do
  BFRS_CODEC_COPIES=$cp timeout -k 10 300 python bench.py $COMMON > "$OUT/regb_${TAG}_$cp.json" \
      2> "$OUT/regb_${TAG}_$cp.err"
  rc=$?; [ $rc -eq 0 ] || { echo "bench copies=$cp rc=$rc"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['crate_api']; print('bench copies', sys.argv[2], 'all_blocks', d['generate_parity_all_blocks_threads']['ms'], 'gp', d['generate_parity']['ms'], 'registered', d.get('registered_inputs'))" "$OUT/regb_${TAG}_$cp.json" $cp
done
