#!/bin/bash
# Gram A/B on the GPU box: RDM parity tests, then the split kernel per launch scheme,
# plus the L2 hit counters of the generation launch.
set -o pipefail
out=gpurun_out/${1:-gram_ab}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "rdm" --timeout 200 --timeout-method thread \
    > $out/pytest_rdm.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest_rdm.log; exit 1; }
tail -2 $out/pytest_rdm.log
timeout -k 10 200 python scripts/probe_gram.py 2>&1 | tee $out/gram_gen.log || exit 1
VISREPS_GRAM_GEN=0 timeout -k 10 200 python scripts/probe_gram.py 2>&1 | tee $out/gram_all.log || exit 1
VISREPS_GRAM_GEN=256 timeout -k 10 200 python scripts/probe_gram.py 2>&1 | tee $out/gram_gen256.log || exit 1
DS=43264 timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $out/pmc -o pmc --output-format csv -- python scripts/probe_gram.py > $out/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
echo done
