#!/bin/bash
# Engine parity tests, then kernel stats of the 14-unit probe with the LDS-DMA B walk
# (default) and without it (VISREPS_ENGINE_DMA=0). Usage: bash scripts/gpu_eng_dma.sh <tag> [pytest files]
set -o pipefail
tag=${1:-dma}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
files=${@:-tests/test_gpu_parity.py tests/test_golden.py tests/test_fullsize.py tests/test_engine_est.py}
timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -5 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; exit 1; }
run() {  # name, env...
  local name=$1; shift
  env "$@" REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  grep engine $out/$name.log
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_countA", "k_join", "k_final", "k_lscan")):
        print("   %-40s calls=%5s avg=%8.1f us" % (n.split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -f $out/$name/p_kernel_trace.csv
}
run dma || exit 1
run nodma VISREPS_ENGINE_DMA=0 || exit 1
