#!/bin/bash
# Bench line (default run, CPU baseline included) + rocprofv3 kernel stats of a short bench,
# the kernels dispatched inside its timed steps (scripts/check_timed_kernels.py), and
# optionally (PMC=1) the FETCH_SIZE / WRITE_SIZE passes of one engine call.
# Usage (from the repo root, via gpurun): bash scripts/gpu_bench.sh [tag]
set -o pipefail
tag=${1:-bench}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 480 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-est-probe --no-extra-legs --no-exact-step \
    > $out/prof.json 2> $out/prof.err || { echo "rocprof failed"; tail -20 $out/prof.err; exit 1; }
python3 scripts/check_timed_kernels.py $out/prof/p_kernel_trace.csv $out/timed_kernels.json || exit 1
rm -f $out/prof/p_kernel_trace.csv
python3 scripts/kstats_summary.py $out/prof/p_kernel_stats.csv 25 2 || true
if [ "${PMC:-0}" = "1" ]; then
  bash scripts/gpu_pmc_engine.sh $tag/pmc || exit 1
fi
