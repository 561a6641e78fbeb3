"""Per-unit HBM bytes of one engine call from the FETCH_SIZE / WRITE_SIZE passes of
scripts/gpu_pmc_engine.sh. FETCH_SIZE x 2 (gfx950: FETCH_SIZE reports half the bytes of
these 128-B row gathers and of wide streams, profiles/r2_fetch_calibration.json).

  python scripts/pmc_engine_summary.py gpurun_out/<tag> <units per call> [n]

The output carries the build (sha256 of the library), N and the engine form, so bench.py
uses it only for the same build and configuration.
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ENGINE = ("k_join", "k_posmap", "k_masks", "k_countA", "k_c0", "k_rankA", "k_lscan", "k_add_base", "k_rankB", "k_tail")


def per_kernel(path):
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("vr::", "")
        if any(k in name for k in ENGINE):
            key = name.split("<")[0]
            agg[key][0] += float(r["Counter_Value"]) * 1024.0  # kB -> B
            agg[key][1] += 1
    return agg


def main(d, units, n=10000):
    f = per_kernel(f"{d}/FETCH_SIZE/p_counter_collection.csv")
    w = per_kernel(f"{d}/WRITE_SIZE/p_counter_collection.csv")
    kern = {}
    total = 0.0
    for k in sorted(set(f) | set(w)):
        fb = 2.0 * f.get(k, [0.0, 0])[0]
        wb = w.get(k, [0.0, 0])[0]
        calls = max(f.get(k, [0, 0])[1], w.get(k, [0, 0])[1])
        kern[k] = {"launches": calls, "fetch_bytes_x2": fb, "write_bytes": wb,
                   "bytes_per_launch": (fb + wb) / max(calls, 1)}
        total += fb + wb
    joined = os.environ.get("JOINED", "0") == "1"
    grid = joined and os.environ.get("GRID", "0") == "1"
    what = (f"the bench's engine path over {units} units (shared joins: vr_engine_posmap4 + vr_engine_join4 "
            "per model plan, then one region-fused vr_bootstrap_spearman_grid_joined call)" if grid else
            f"{units} units (shared joins: vr_engine_posmap4 + vr_engine_join4 per model plan, then one "
            "vr_bootstrap_spearman_multi_joined call per region)" if joined else
            f"one {units}-unit vr_bootstrap_spearman_multi call")
    out = {"source": (f"rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE (separate passes) over {what} on the bench "
                      "RDMs (scripts/gpu_pmc_engine.sh); FETCH_SIZE x 2 (gfx950 correction)"),
           "joined": joined, "grid": grid,
           "units_per_call": units, "call_bytes": total, "bytes_per_unit": total / units,
           "kernels": kern, "n": n, "est": os.environ.get("VISREPS_ENGINE_EST") != "0",
           "build_id": build_id()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    from visreps_amd._lib import build_id

    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 10000)
