#!/bin/bash
# Radix sort (sort.hip) check + A/B: the GPU parity file (unless SKIP_TESTS), then
# scripts/probe_sort.py with the default library and each abl/<name>.so, twice, and the
# rocprofv3 kernel stats of one run per library.   bash scripts/gpu_sort_ab.sh <names...>
set -o pipefail
out=gpurun_out/r3sort
mkdir -p $out
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $out/pytest.log
for r in 1 2; do
  timeout -k 10 120 python scripts/probe_sort.py || exit 1
  for v in "$@"; do VISREPS_AMD_LIB=$PWD/abl/$v.so timeout -k 10 120 python scripts/probe_sort.py || exit 1; done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/default -o p --output-format csv -- python scripts/probe_sort.py > /dev/null 2>&1 || exit 1
for v in "$@"; do
  VISREPS_AMD_LIB=$PWD/abl/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/$v -o p --output-format csv -- python scripts/probe_sort.py > /dev/null 2>&1 || exit 1
done
for v in default "$@"; do
  python3 - $out/$v/p_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "vr::" in r["Name"]:
        print(sys.argv[2], r["Name"].split("(")[0], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
