#!/bin/bash
# Half-word transpose check: engine + Kendall parity tests, then Kendall level times and the
# region-fused grid probe for the default build and the 64-bit-stage build (abl/x1.so).
set -o pipefail
tag=${1:-xp}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_engine_est.py tests/test_kendall.py tests/test_gpu_parity.py > $out/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
bash scripts/gpu_kendall_levels.sh $tag/klv abl/x1.so || exit 1
bash scripts/gpu_grid_ab.sh $tag/grid abl/x1.so || exit 1
rm -f $out/grid/*/p_kernel_trace.csv
