"""Summary of one gpu_gram_pmc_e.sh pass: per wide-Gram dispatch the MFMA-busy fraction of
the SQ-busy cycles and of 1024 SIMDs x duration x 2.4 GHz, the clock the dispatch ran at
(GRBM_GUI_ACTIVE / 8 XCDs / duration, MI355X_MICROARCH.md 'DVFS give-back'), and the wait
fractions. Usage: python scripts/gram_pmc_summary.py <p_counter_collection.csv> <kernel> <D>"""
import collections
import csv
import json
import sys

rows = collections.defaultdict(dict)
with open(sys.argv[1]) as f:
    cols = f.readline().strip()
if "Counter_Name" not in cols:
    sys.exit("unexpected columns: " + cols)
meta = {}
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if "k_gram3e" not in name and "k_gram3p" not in name:
        continue
    d = int(r["Dispatch_Id"])
    rows[d][r["Counter_Name"]] = rows[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ts = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e9 if "End_Timestamp" in r else float("nan")
    meta[d] = (name.split("(")[0].replace("vr::", ""), ts)
out = []
for d in sorted(rows):
    c, (name, sec) = rows[d], meta[d]
    w = max(c.get("SQ_WAVE_CYCLES", 0.0), 1.0)
    out.append({"dispatch": d, "kernel": name, "ms": round(sec * 1e3, 3),
                "clock_ghz": round(c.get("GRBM_GUI_ACTIVE", 0.0) / 8 / sec / 1e9, 3),
                "mfma_util_nominal_2p4": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * sec * 2.4e9), 4),
                "mfma_util_at_clock": round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c.get("GRBM_GUI_ACTIVE", 1.0) / 8), 4),
                "wait_inst_frac": round(c["SQ_WAIT_INST_ANY"] / w, 4), "wait_any_frac": round(c["SQ_WAIT_ANY"] / w, 4),
                "lds_bank_conflict_over_lds": round(c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_ACTIVE_INST_LDS"], 1.0), 4)})
print(json.dumps({"kernel_form": sys.argv[2], "D": int(sys.argv[3]), "dispatches": out}))
