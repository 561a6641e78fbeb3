#!/bin/bash
# Default build vs the previous in-tree build (abl/prev.so): engine probe kernel stats, twice
# each, interleaved. Usage (via gpurun): bash scripts/gpu_prev_ab.sh <tag>
set -o pipefail
tag=${1:-prevab}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
run() {  # name, env...
  local name=$1; shift
  env "$@" REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep engine $out/$name.log
  rm -f $out/$name/p_kernel_trace.csv
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB")):
        print("   %-48s calls=%5s avg=%8.1f us" % (n.split("(")[0][-48:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
run new1 || exit 1
run prev1 ALT_LIB=$PWD/abl/prev.so || exit 1
run new2 || exit 1
run prev2 ALT_LIB=$PWD/abl/prev.so || exit 1
