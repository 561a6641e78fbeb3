#!/bin/bash
# Kendall per-stream walk times: kernel trace of the 1001-subset unit (probe_kendall.py),
# then kendall_levels.py. Usage (via gpurun): bash scripts/gpu_kendall_levels.sh <tag> [lib.so ...]
set -o pipefail
tag=${1:-klv}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" CASES=unit timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_kendall.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep unit $out/$name.log
  python3 scripts/kendall_levels.py $out/$name/p_kernel_trace.csv 16 | tee $out/$name.levels
  python3 scripts/kstats_summary.py $out/$name/p_kernel_stats.csv 14 | tee $out/$name.kstats
  rm -f $out/$name/p_kernel_trace.csv
}
run default || exit 1
for lib in "$@"; do
  run $(basename $lib .so) VISREPS_AMD_LIB=$PWD/$lib || exit 1
done
