#!/bin/bash
# Round 6: where the exact form's time goes -- the 56-unit joined probe with every pass exact
# (VISREPS_ENGINE_EST=0), kernel stats, beside the default grid path.
set -o pipefail
out=gpurun_out/r6i
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
for mode in grid; do
  if [ $mode = exact ]; then E=0; G=0; else E=1; G=1; fi
  VISREPS_ENGINE_EST=$E JOINED=1 GRID=$G REPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/$mode -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$mode.log 2>&1 || { echo "probe $mode failed"; tail -5 $out/$mode.log; exit 1; }
  grep engine $out/$mode.log
  python3 scripts/kstats_summary.py $out/$mode/p_kernel_stats.csv 16 1 | grep -v "naive\|igemm\|Cijk\|conv\|Conv\|gram\|transpose\|BatchNorm\|Im2d" || true
  rm -f $out/$mode/p_kernel_trace.csv
done
