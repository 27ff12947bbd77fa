"""Per-dispatch shader clock and pipe utilisation from one rocprofv3 --pmc pass
that includes GRBM_GUI_ACTIVE (tools/pmc_kernel.py launch loop).

clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration; busy% = counter / 256
CUs / (GRBM_GUI_ACTIVE / 8), the MI355X_MICROARCH.md derived-metric form.
usage: python tools/pmc_clock.py gpurun_out/pmc_TAG_v*/pmc_counter_collection.csv"""
import collections
import csv
import statistics
import sys

for f in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for r in csv.DictReader(open(f)):
        if ("gf_apply" not in r["Kernel_Name"] and "gf_encode" not in r["Kernel_Name"]) or int(r["Grid_Size"]) < 1000000:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(per, key=int)
    steady = ids[len(ids) // 2:]  # second half: past the clock ramp
    g = {i: per[i]["GRBM_GUI_ACTIVE"] / 8 for i in steady}
    out = {"dispatches": len(ids),
           "ms": round(statistics.median(dur[i] for i in steady) / 1e6, 4),
           "clock_GHz": round(statistics.median(g[i] / dur[i] for i in steady), 3),
           "first_clock_GHz": round(per[ids[0]]["GRBM_GUI_ACTIVE"] / 8 / dur[ids[0]], 3)}
    for name, key in (("VALUbusy%", "SQ_ACTIVE_INST_VALU"), ("LDSactive%", "SQ_LDS_IDX_ACTIVE"),
                      ("LDSconflict%", "SQ_LDS_BANK_CONFLICT")):
        if any(key in per[i] for i in steady):
            out[name] = round(statistics.median(100 * per[i][key] / 256 / g[i] for i in steady), 1)
    print(f.split("/")[-2], out)
