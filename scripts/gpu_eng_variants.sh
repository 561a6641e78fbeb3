#!/bin/bash
# Engine kernel timings per library build (rocprofv3 kernel stats of the 14-unit probe).
# Usage: bash scripts/gpu_eng_variants.sh <tag> [lib.so ...]   (default build first, then
# the default build in the exact chunk-base form, then each alternative build)
set -o pipefail
tag=${1:-eng}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" REPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/${PROBE:-probe_engine_bench.py} > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep engine $out/$name.log
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_countA", "k_join")):
        print("   %-40s calls=%5s avg=%8.1f us" % (n.split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
run default || exit 1
run exact VISREPS_ENGINE_EST=0 || exit 1
for lib in "$@"; do
  run $(basename $lib .so) ALT_LIB=$PWD/$lib || exit 1
done
# masks read from L2 instead of LDS, default build and the 512-thread build
run default_gmask VISREPS_ENGINE_MASKS=global || exit 1
[ -f altlib/lib_t512.so ] && { run t512_gmask VISREPS_ENGINE_MASKS=global ALT_LIB=$PWD/altlib/lib_t512.so || exit 1; }
