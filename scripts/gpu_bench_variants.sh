#!/bin/bash
# Engine kernel timings inside the bench (rocprofv3 kernel stats of one timed step) per
# library build / env. Usage: bash scripts/gpu_bench_variants.sh <tag> "name:ENV=V,ENV2=V2" ...
set -o pipefail
tag=${1:-bv}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $out/$name.json 2> $out/$name.err \
      || { echo "$name failed"; tail -5 $out/$name.err; exit 1; }
  python3 - "$out/$name/p_kernel_stats.csv" "$name" "$out/$name.json" <<'PY'
import csv, sys, json
line = [l for l in open(sys.argv[3]) if l.startswith("{")]
v = json.loads(line[-1])["value"] if line else None
print(f"{sys.argv[2]}: step {v} s")
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_countA", "k_join", "k_gram3w")):
        print("   %-40s calls=%5s avg=%8.1f us total=%8.1f ms" % (n.split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
  rm -f $out/$name/p_kernel_trace.csv
done
