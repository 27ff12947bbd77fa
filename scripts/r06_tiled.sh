#!/bin/bash
# Round 6: tile-major shard sets vs the product's row layout, v76, same process,
# three copies of each layout interleaved in allocation order (placement).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/tiled
mkdir -p "$OUT"
L=${LAYOUTS:-12288,0a,12288#2,0a#2,12288#3,0a#3,0t,0t#2}
timeout -k 10 300 python3 tools/kbench.py --variants ${VARIANTS:-76} --stagger "$L" --rounds 3 --iters 10 \
    > "$OUT/kb_enc.json" 2> "$OUT/kb_enc.err"
rc=$?; echo "enc rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/kb_enc.err"; exit $rc; }
timeout -k 10 300 python3 tools/kbench.py --variants ${VARIANTS:-76} --stagger "$L" --rounds 3 --iters 10 --decode \
    > "$OUT/kb_dec.json" 2> "$OUT/kb_dec.err"
rc=$?; echo "dec rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/kb_dec.err"; exit $rc; }
python3 - <<'PY'
import json
for f in ("enc", "dec"):
    d = json.load(open(f"gpurun_out/tiled/kb_{f}.json"))
    print(f, {k: v["ms"] for k, v in d.items() if isinstance(v, dict) and "ms" in v})
PY
