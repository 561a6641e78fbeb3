#!/bin/bash
# bench.py under rocprofv3 kernel stats (steps/warmup from args), then the plain bench line
# Usage: bash scripts/gpu_bench_prof.sh <tag> [steps] [warmup] [extra env...]
set -o pipefail
tag=${1:-bp}; steps=${2:-2}; warmup=${3:-1}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv \
    -- python bench.py --steps $steps --warmup $warmup --no-cpu-baseline > $out/bench_prof.json 2> $out/bench_prof.err \
    || { echo "profiled bench failed"; tail -20 $out/bench_prof.err; exit 1; }
rm -f $out/prof/p_kernel_trace.csv
python3 scripts/kstats_summary.py $out/prof/p_kernel_stats.csv 30 $((steps + warmup)) || true
cat $out/bench_prof.json
