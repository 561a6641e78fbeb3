#!/bin/bash
# SQ counters of the engine kernels on the bench RDMs (probe_engine_bench.py, REPS=1), one
# rocprofv3 --pmc pass per configuration. Usage: bash scripts/gpu_eng_pmc.sh <tag> "name:ENV=V" ...
set -o pipefail
tag=${1:-pmc}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"}
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } REPS=1 timeout -s KILL 240 rocprofv3 --pmc $CTRS -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; exit 1; }
  python3 - "$out/$name/p_counter_collection.csv" "$name" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in ("k_rankB", "k_rankA", "k_countA"):
        if k in n:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
print(sys.argv[2])
for k, d in agg.items():
    calls = max(cnt[(k, c)] for c in d)
    print("  %-9s calls=%d  " % (k, calls) + "  ".join("%s=%.4g" % (c.replace("SQ_", ""), v / calls) for c, v in sorted(d.items())))
PY
done
