#!/bin/bash
# Round-3 parity additions on the GPU: full-size CPU-oracle parity of the bench points,
# TVSD / THINGS / ridge at their stated sizes, and the small-n end-to-end margins.
set -o pipefail
tag=${1:-r3_parity}
out=gpurun_out/$tag
mkdir -p $out
export VISREPS_MARGINS=$out/parity_margins.jsonl
rm -f $VISREPS_MARGINS
timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -m gpu \
    tests/test_benchsize.py::test_bench_point_vs_cpu_oracle tests/test_tvsd.py tests/test_drivers.py \
    tests/test_encoding.py::test_ridge_cv_full_size_matches_closed_form tests/test_eval.py tests/test_phase1.py \
    > $out/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $out/pytest.log | tail -30
cat $VISREPS_MARGINS
exit $rc
