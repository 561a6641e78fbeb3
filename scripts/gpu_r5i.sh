#!/bin/bash
# Grid engine: its GPU tests, then the 56-unit joined probe per region vs region-fused (kernel stats).
set -o pipefail
tag=${1:-r5i}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_engine_est.py \
    > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for g in 0 1; do
  JOINED=1 GRID=$g REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/g$g -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/g$g.log 2>&1 || { echo "probe g$g failed"; tail -5 $out/g$g.log; exit 1; }
  grep engine $out/g$g.log
  python3 - "$out/g$g/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_join4", "k_full_corr", "k_tail")):
        print("   %-44s calls=%5s avg=%8.1f us total=%8.1f ms" % (n.split("(")[0][-44:], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
done
