#!/bin/bash
# Prefetching EST 3/4 B walk (default build) vs the per-window walk (abl/xw0.so, -DVR_XWIN=0,
# with the join's streamed low ends as before, VISREPS_ENGINE_LO_JOIN=1): kernel stats of the
# 14-unit engine probe. Usage (via gpurun): bash scripts/gpu_xwin_ab.sh <tag>
set -o pipefail
tag=${1:-xwin}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
run() {  # name, env...
  local name=$1; shift
  env "$@" REPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep engine $out/$name.log
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_join")):
        print("   %-40s calls=%5s avg=%8.1f us" % (n.split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
run xwin || exit 1
run perwin ALT_LIB=$PWD/abl/xw0.so VISREPS_ENGINE_LO_JOIN=1 || exit 1
run perwin_lo0 ALT_LIB=$PWD/abl/xw0.so VISREPS_ENGINE_LO_JOIN=0 || exit 1
