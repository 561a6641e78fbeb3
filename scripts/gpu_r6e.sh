#!/bin/bash
# Round 6: engine tests (EST 1 fallback only with L2 masks), 73k plan-free statistics with the
# default sort tiles and 8192-key tiles (abl/rs32.so), kernel stats of each.
set -o pipefail
out=gpurun_out/r6e
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_engine_est.py -m gpu -k "structured" > $out/engine_est.log 2>&1 || { tail -40 $out/engine_est.log; exit 1; }
tail -3 $out/engine_est.log
for lib in default rs32; do
  if [ $lib = default ]; then unset ALT_LIB; else export ALT_LIB=$PWD/abl/$lib.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$lib -o p --output-format csv -- python scripts/probe_full73k.py > $out/full73k_$lib.log 2>&1 || { tail -20 $out/full73k_$lib.log; exit 1; }
  cat $out/full73k_$lib.log | grep -v amdgpu.ids
  python3 scripts/kstats_summary.py $out/prof_$lib/p_kernel_stats.csv 14 1 || true
  rm -f $out/prof_$lib/p_kernel_trace.csv
done
