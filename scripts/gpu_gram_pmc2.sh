#!/bin/bash
# Gram probe under separate rocprofv3 --pmc passes: HBM bytes (FETCH_SIZE, WRITE_SIZE), L2
# hit/miss and MFMA busy, for k_gram3w at the bench's widths (N = 10k).
set -o pipefail
tag=${1:-gpmc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for spec in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "l2:TCC_HIT_sum TCC_MISS_sum" "mfma:SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  name=${spec%%:*}; ctr=${spec#*:}
  DS=290400,43264 REPS=1 timeout -s KILL 120 rocprofv3 --pmc $ctr -d $out/$name -o p --output-format csv \
      -- python scripts/probe_gram.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; exit 1; }
done
python3 - $out <<'PY'
import csv, sys, collections
out = sys.argv[1]
for name in ["fetch", "write", "l2", "mfma"]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{out}/{name}/p_counter_collection.csv")):
        if "k_gram" in r["Kernel_Name"]:
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(name, k, {c: [round(v / 1e6, 3) for v in vs] for c, vs in d.items()})
PY
