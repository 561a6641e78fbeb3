#!/bin/bash
# Wide (256 x 256) split Gram on the GPU box: RDM/Gram parity tests, then timings wide vs 128.
set -o pipefail
out=gpurun_out/${1:-gram_wide}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_encoding.py -m gpu -x -q --tb=short -k "rdm or gram" --timeout 200 --timeout-method thread \
    > $out/pytest_rdm.log 2>&1 || { echo "pytest failed"; tail -c 3000 $out/pytest_rdm.log; exit 1; }
tail -2 $out/pytest_rdm.log
timeout -k 10 200 python scripts/probe_gram.py 2>&1 | tee $out/gram_wide.log || exit 1
VISREPS_GRAM_WIDE=0 timeout -k 10 200 python scripts/probe_gram.py 2>&1 | tee $out/gram_128.log || exit 1
CASES=0 timeout -k 10 200 python scripts/probe_scale.py 2>&1 | tee $out/scale_wide.log || exit 1
