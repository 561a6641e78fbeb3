#!/bin/bash
# Engine A/B: kernel stats of the 14-unit probe for the default build and each alternative
# library. Usage (via gpurun): bash scripts/gpu_eng_ab.sh <tag> [lib.so ...]
set -o pipefail
tag=${1:-engab}; shift
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
run default || exit 1
for lib in "$@"; do
  run $(basename $lib .so) ALT_LIB=$PWD/$lib || exit 1
done
