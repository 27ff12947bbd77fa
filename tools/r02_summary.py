"""Summary of one scripts/r02_variants.sh / r02_pmc.sh session (gpurun_out/*TAG*):
kbench medians per variant and direction, and per-variant SQ counter ratios."""
import collections
import csv
import glob
import json
import statistics
import sys

tag = sys.argv[1]
for f in (f"gpurun_out/kb_{tag}_enc.log", f"gpurun_out/kb_{tag}_dec.log"):
    try:
        s = open(f).read()
        d = json.loads(s[s.index("{"):])
        print(f, {k: v["ms"] for k, v in d.items() if isinstance(v, dict)})
    except Exception as e:  # noqa: BLE001
        print(f, "n/a", e)
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}_v*/pmc_counter_collection.csv")):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "gf_apply" not in r["Kernel_Name"] or int(r["Grid_Size"]) < 1000000:
            continue
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = {c: statistics.median(d.values()) for c, d in per.items()}
    out = {k: f"{x:.4g}" for k, x in sorted(v.items())}
    if "GRBM_GUI_ACTIVE" in v:
        g = v["GRBM_GUI_ACTIVE"] / 8
        for name, key in (("VALUbusy%", "SQ_ACTIVE_INST_VALU"), ("LDSactive%", "SQ_LDS_IDX_ACTIVE"),
                          ("LDSconflict%", "SQ_LDS_BANK_CONFLICT")):
            if key in v:
                out[name] = round(100 * v[key] / 256 / g, 1)
    print(f.split("/")[1], out)
