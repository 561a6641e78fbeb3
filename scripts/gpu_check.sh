#!/bin/bash
# One GPU-box session: parity suite, bench line, rocprofv3 kernel stats of the bench.
# Usage (from the repo root, via gpurun): bash scripts/gpu_check.sh [tag]
set -o pipefail
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > $out/pytest_gpu.log 2>&1 || { echo "pytest failed: $?"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline \
    > $out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $out/prof.log; exit 1; }
find $out/prof -name '*stats*' | head
