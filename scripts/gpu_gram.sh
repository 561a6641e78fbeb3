#!/bin/bash
# Gram check on the GPU box: RDM parity tests, then split vs fp32 kernel timings.
set -o pipefail
out=gpurun_out/${1:-gram}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rdm" --timeout 200 --timeout-method thread \
    > $out/pytest_rdm.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_rdm.log; exit 1; }
tail -2 $out/pytest_rdm.log
timeout -k 10 200 python scripts/probe_gram.py 2>&1 | tee $out/gram_split.log || exit 1
VISREPS_GRAM=fp32 DS=43264 timeout -k 10 200 python scripts/probe_gram.py 2>&1 | tee $out/gram_fp32.log || exit 1
