#!/bin/bash
# TB row stores: nontemporal (default build) vs default policy (abl/tbnt0.so,
# -DVR_TB_STORE_NT=0), kernel stats of the 14-unit engine probe; plus the row-write
# microbench (scripts/microbench_scatter.hip, built on the box). Usage: bash scripts/gpu_nt_ab.sh <tag>
set -o pipefail
tag=${1:-ntab}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
hipcc --offload-arch=gfx950 -O3 scripts/microbench_scatter.hip -o /tmp/mb_scatter && timeout -k 10 120 /tmp/mb_scatter > $out/mb.log 2>&1 && cat $out/mb.log || exit 1
for v in default tbnt0; do
  extra=""; [ $v = tbnt0 ] && extra="ALT_LIB=$PWD/abl/tbnt0.so"
  env $extra REPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$v -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$v.log 2>&1 || { echo "$v failed"; tail -5 $out/$v.log; exit 1; }
  grep engine $out/$v.log
  python3 - "$out/$v/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_join")):
        print("   %-48s calls=%5s avg=%8.1f us" % (n.split("(")[0][-48:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
