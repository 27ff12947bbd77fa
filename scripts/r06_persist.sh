#!/bin/bash
# Round 6: v110 (persistent workgroups, ring carried across T tiles) vs v76,
# one process, three copies of the row layout (placement), encode and decode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/persist
mkdir -p "$OUT"
L=${LAYOUTS:-12288,12288#2,12288#3}
V=${VARIANTS:-76,110t2,110t4}
for io in enc dec; do
  flag=""; [ $io = dec ] && flag="--decode"
  timeout -k 10 300 python3 tools/kbench.py --variants "$V" --stagger "$L" --rounds 3 --iters 10 $flag \
      > "$OUT/kb_$io.json" 2> "$OUT/kb_$io.err"
  rc=$?; echo "$io rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/kb_$io.err"; exit $rc; }
done
python3 - <<'PY'
import json
for f in ("enc", "dec"):
    d = json.load(open(f"gpurun_out/persist/kb_{f}.json"))
    print(f, {k: v["ms"] for k, v in d.items() if isinstance(v, dict) and "ms" in v})
PY
