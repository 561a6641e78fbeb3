"""HBM traffic per engine call / per Gram launch from the rocprofv3 --pmc passes of
scripts/gpu_pmc.sh (FETCH_SIZE and WRITE_SIZE, kB). Writes a JSON summary.

  python scripts/pmc_traffic.py gpurun_out/<tag> [units per call] > profiles/<name>.json
"""
import collections
import csv
import json
import sys

ENGINE = ("k_join", "k_masks", "k_countA", "k_c0", "k_rankA", "k_lscan", "k_add_base", "k_rankB", "k_tail")


def load(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)  # kB -> B
    return agg


def main(d):
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), raw counter "
                     "values x 1024 B; no gfx950 correction applied (see DESIGN.md)"}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        eng = load(f"{d}/eng_{c}/p_counter_collection.csv")
        per_kernel = {}
        total = 0.0
        for name, vals in eng.items():
            short = name.split("(")[0].replace("void ", "").replace("vr::", "")
            if any(k in short for k in ENGINE):
                s = sum(vals)
                total += s
                per_kernel[short] = per_kernel.get(short, 0.0) + s
        out[f"engine_call_{c}"] = total  # one unit (REPS=1): all kernels of the call
        out[f"engine_kernels_{c}"] = per_kernel
        gram = load(f"{d}/gram_{c}/p_counter_collection.csv")
        g = [v for n, vals in gram.items() if "k_gram" in n for v in vals]
        out[f"gram_launch_{c}"] = sum(g) / len(g) if g else None
    out["engine_call_bytes"] = out["engine_call_FETCH_SIZE"] + out["engine_call_WRITE_SIZE"]
    out["gram_launch_bytes"] = out["gram_launch_FETCH_SIZE"] + out["gram_launch_WRITE_SIZE"]
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    out["engine_units_per_call"] = nb
    out["engine_unit_bytes"] = out["engine_call_bytes"] / nb
    out["gram_config"] = "N=10000, D=43264 fp32 input (split kernel: bf16 hi/lo records)"
    out["engine_config"] = (f"N=10000, {nb} units per call (one shared neural plan), 1001 subsets "
                            "(point + 1000 bootstrap), 16 passes")
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])  # argv[2]: units per engine call
