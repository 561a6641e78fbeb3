#!/bin/bash
# B-walk work-queue segments per wave on the 14-unit engine probe: the default build and
# abl/segsb.so (the VISREPS_ENGINE_SEGS_B switch) at 1 and 4. Usage: bash scripts/gpu_segsb_probe.sh <tag>
set -o pipefail
tag=${1:-segsbp}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
run() {
  local name=$1; shift
  env "$@" REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep engine $out/$name.log
  rm -f $out/$name/p_kernel_trace.csv
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankB", "k_tail")):
        print("   %-48s calls=%5s avg=%8.1f us" % (n.split("(")[0][-48:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
run default || exit 1
run segsb4 ALT_LIB=$PWD/abl/segsb.so VISREPS_ENGINE_SEGS_B=4 || exit 1
run segsb1 ALT_LIB=$PWD/abl/segsb.so VISREPS_ENGINE_SEGS_B=1 || exit 1
run segsb4b ALT_LIB=$PWD/abl/segsb.so VISREPS_ENGINE_SEGS_B=4 || exit 1
