#!/bin/bash
# Kernel stats + checksum of the 14-unit engine probe for LDS-DMA B-walk builds.
# Usage: bash scripts/gpu_eng_dma_variants.sh <tag> name[:lib.so] ...  ("nodma" = VISREPS_ENGINE_DMA=0)
set -o pipefail
tag=${1:-dmav}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; lib=${spec#*:}; [ "$lib" = "$spec" ] && lib=""
  envs="REPS=2"
  [ -n "$lib" ] && envs="$envs ALT_LIB=$PWD/$lib"
  [ "$name" = "nodma" ] && envs="$envs VISREPS_ENGINE_DMA=0"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; exit 1; }
  echo "== $name: $(grep engine $out/$name.log)"
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB")):
        print("   %-40s calls=%5s avg=%8.1f us" % (n.split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -f $out/$name/p_kernel_trace.csv
done
