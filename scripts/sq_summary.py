"""Per-kernel SQ summary of a rocprofv3 --pmc pass (p_counter_collection.csv): for every
dispatch of kernels whose name matches a regex, the counters summed over the dispatch, then
averaged over dispatches of the same kernel, with fractions of SQ_WAVE_CYCLES / SQ_BUSY_CYCLES
and the clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).
Usage: python scripts/sq_summary.py <csv> <kernel-regex>"""
import collections
import csv
import json
import re
import sys

pat = re.compile(sys.argv[2])
per = collections.defaultdict(dict)
meta = {}
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if not pat.search(name):
        continue
    d = int(r["Dispatch_Id"])
    per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    meta[d] = (name.split("(")[0].replace("void ", "").replace("vr::", ""),
               (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e9)
groups = collections.defaultdict(list)
for d, c in per.items():
    groups[meta[d][0]].append((meta[d][1], c))
out = {}
for k, lst in groups.items():
    n = len(lst)
    avg = collections.defaultdict(float)
    for sec, c in lst:
        for key, v in c.items():
            avg[key] += v / n
        avg["_sec"] += sec / n
    w = max(avg.get("SQ_WAVE_CYCLES", 0.0), 1.0)
    b = max(avg.get("SQ_BUSY_CYCLES", 0.0), 1.0)
    e = {"dispatches": n, "avg_us": round(avg["_sec"] * 1e6, 1)}
    if "GRBM_GUI_ACTIVE" in avg:
        e["clock_ghz"] = round(avg["GRBM_GUI_ACTIVE"] / 8 / avg["_sec"] / 1e9, 3)
    for key in sorted(avg):
        if key.startswith("SQ_") and key not in ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
            e[key] = round(avg[key])
            e[key + "/wave_cycles"] = round(avg[key] / w, 4)
    e["SQ_WAVE_CYCLES"] = round(w)
    e["SQ_BUSY_CYCLES"] = round(b)
    out[k] = e
print(json.dumps(out, indent=1))
