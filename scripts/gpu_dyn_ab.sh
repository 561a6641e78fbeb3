#!/bin/bash
# EST work-queue segments (default build: B walk one segment per wave, A side 4) vs the
# round-4 static split (abl/static.so), and the default build with 2 / 1 A segments per wave.
# Usage (via gpurun): bash scripts/gpu_dyn_ab.sh <tag>
set -o pipefail
tag=${1:-dyn}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
run() {  # name, env...
  local name=$1; shift
  env "$@" REPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep engine $out/$name.log
  rm -f $out/$name/p_kernel_trace.csv
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_join", "k_countA", "k_tail")):
        print("   %-48s calls=%5s avg=%8.1f us" % (n.split("(")[0][-48:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
run queueA4 || exit 1
run static ALT_LIB=$PWD/abl/static.so || exit 1
run queueA2 VISREPS_ENGINE_SEGS_A=2 || exit 1
run queueA1 VISREPS_ENGINE_SEGS_A=1 || exit 1
