#!/bin/bash
# Per-walk transpose forms: engine + Kendall parity, Kendall stream times + kernel stats,
# grid probe for the default build vs the A-walk alternatives (abl/a1.so, abl/a2.so).
set -o pipefail
tag=${1:-xp2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_engine_est.py tests/test_kendall.py > $out/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
bash scripts/gpu_kendall_levels.sh $tag/klv || exit 1
bash scripts/gpu_grid_ab.sh $tag/grid abl/a1.so abl/a2.so || exit 1
rm -f $out/grid/*/p_kernel_trace.csv
