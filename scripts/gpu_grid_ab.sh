#!/bin/bash
# Region-fused engine A/B: the 56-unit joined probe (GRID=1) for the default build and each
# alternative library, kernel stats. Usage (via gpurun): bash scripts/gpu_grid_ab.sh <tag> [lib.so ...]
set -o pipefail
tag=${1:-gridab}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
run() {  # name, env...
  local name=$1; shift
  env "$@" JOINED=1 GRID=1 REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep engine $out/$name.log
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_full_corr")):
        print("   %-44s calls=%5s avg=%8.1f us total=%8.1f ms" % (n.split("(")[0][-44:], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
}
run default || exit 1
for lib in "$@"; do
  run $(basename $lib .so) ALT_LIB=$PWD/$lib || exit 1
done
