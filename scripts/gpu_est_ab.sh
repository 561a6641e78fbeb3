#!/bin/bash
# EST pass-form A/B on the bench RDMs (probe_engine_bench.py under rocprofv3 kernel stats,
# each EST form checked bit for bit against the exact form in the same process), then the
# EST parity tests. Usage: bash scripts/gpu_est_ab.sh <tag> [name:lib.so | name:VAR=value ...]
set -o pipefail
tag=${1:-estab}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" REPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/$name -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }
  echo "== $name: $(grep engine $out/$name.log)"
  python3 - "$out/$name/p_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_rankA", "k_rankB", "k_countA", "k_join")):
        print("   %-60s calls=%5s avg=%8.1f us" % (n.split("(")[0][-60:], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -f $out/$name/p_kernel_trace.csv
}
run default VISREPS_ENGINE_EST=1 || exit 1
for spec in "$@"; do
  arg=${spec#*:}
  if [[ "$arg" == *=* ]]; then
    run ${spec%%:*} VISREPS_ENGINE_EST=1 "$arg" || exit 1
  else
    run ${spec%%:*} VISREPS_ENGINE_EST=1 ALT_LIB=$PWD/$arg || exit 1
  fi
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_est.py \
    > $out/pytest_est.log 2>&1; echo "pytest rc=$?: $(tail -1 $out/pytest_est.log)"
