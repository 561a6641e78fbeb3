#!/bin/bash
# Round-2 GPU session: selected pytest files, then optionally the bench and its rocprof stats.
# Usage (via gpurun, from the repo root): bash scripts/gpu_r2.sh <tag> "<pytest files>" [bench]
set -o pipefail
tag=${1:-run}
tests=${2:-tests}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
if [ "$tests" != "none" ]; then
  timeout -k 10 900 python -u -m pytest $tests -m gpu -x -v --timeout 240 --timeout-method thread \
      > $out/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; grep -E "PASS|FAIL|Error|error" $out/pytest_gpu.log | tail -40; exit 1; }
  grep -cE "PASSED" $out/pytest_gpu.log; tail -3 $out/pytest_gpu.log
fi
if [ "$3" == "bench" ]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 2 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
  cat $out/bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline \
      > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $out/prof.log; exit 1; }
  find $out/prof -name '*stats*' | head
fi
