#!/bin/bash
# bench-size parity tests, then the bench (full default run incl. CPU baseline)
set -o pipefail
out=gpurun_out/r2b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_benchsize.py -m gpu -v --timeout 300 --timeout-method thread \
    > $out/pytest_benchsize.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" $out/pytest_benchsize.log | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
timeout -k 10 600 python bench.py --steps 3 --warmup 2 > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
