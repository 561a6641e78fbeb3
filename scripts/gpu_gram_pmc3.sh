#!/bin/bash
# SQ counters of the wide Gram kernels (probe_gram.py, N=10k, D=43264), one pass per kernel form.
set -o pipefail
out=gpurun_out/${1:-gram_pmc3}
mkdir -p $out
export TMPDIR=/tmp
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"
for pipe in 1 0; do
  VISREPS_GRAM_PIPE=$pipe DS=43264 timeout -s KILL 90 rocprofv3 --pmc $C -d $out/p$pipe -o p --output-format csv \
      -- python scripts/probe_gram.py > $out/p$pipe.log 2>&1 || { echo "pmc pipe=$pipe failed"; tail -5 $out/p$pipe.log; exit 1; }
  python3 - $out/p$pipe/p_counter_collection.csv $pipe <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "k_gram3" in r["Kernel_Name"] and ("k_gram3p" in r["Kernel_Name"] or "k_gram3w" in r["Kernel_Name"]):
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
print("pipe=" + sys.argv[2], {k: "%.4g" % (v / max(cnt[k], 1)) for k, v in sorted(agg.items())})
w = agg["SQ_WAVE_CYCLES"]
print("  MFMA_BUSY/BUSY_CYCLES %.3f  WAIT_INST_ANY/WAVE %.3f  WAIT_ANY/WAVE %.3f  LDS_ACTIVE/WAVE %.3f  BANK_CONFLICT/LDS_ACTIVE %.3f" % (
    agg["SQ_VALU_MFMA_BUSY_CYCLES"] / max(agg["SQ_BUSY_CYCLES"], 1), agg["SQ_WAIT_INST_ANY"] / w, agg["SQ_WAIT_ANY"] / w,
    agg["SQ_ACTIVE_INST_LDS"] / w, agg["SQ_LDS_BANK_CONFLICT"] / max(agg["SQ_ACTIVE_INST_LDS"], 1)))
PY
done
