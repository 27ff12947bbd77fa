"""Prints ms / GB/s per variant from tools/kbench.py logs."""
import json
import sys

for f in sys.argv[1:]:
    t = open(f).read()
    d = json.loads(t[t.find("{"):])
    print("==", f)
    for k, v in d.items():
        if isinstance(v, dict) and "ms" in v:
            print(f"  {k:32s} {v['ms']:.4f} ms {v['GBps']:8.1f} GB/s {v.get('all_ms', '')}")
