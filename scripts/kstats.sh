#!/bin/bash
# per-kernel stats of a probe under rocprofv3: kstats.sh <tag> <python script> [ALT_LIB]
set -o pipefail
tag=$1; script=$2; lib=$3
mkdir -p gpurun_out/ks
export TMPDIR=/tmp
ALT_LIB=$lib REPS=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ks/$tag -o k --output-format csv -- python $script > gpurun_out/ks/$tag.log 2>&1 || { tail gpurun_out/ks/$tag.log; exit 1; }
f=$(find gpurun_out/ks/$tag -name 'k_kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:9.1f} pct={r['Percentage']}")
PY
