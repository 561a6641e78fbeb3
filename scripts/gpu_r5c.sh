#!/bin/bash
# Engine tests + engine A/B probe (default, VALU / SALU slope probes).
set -o pipefail
tag=${1:-r5c}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_engine_est.py tests/test_gpu_parity.py \
    > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash scripts/gpu_eng_ab.sh $tag/eng abl/xp0.so abl/xp64.so abl/xp128.so || exit 1
