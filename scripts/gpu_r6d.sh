#!/bin/bash
# Round 6: bootstrap beyond the rank plans (bootstrap_full), one-product bf16 Gram, compute_rsa,
# and the configs[4] ViT RDM parity at N = 50k on the one-product kernel.
set -o pipefail
out=gpurun_out/r6d
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST VISREPS_MARGINS=$PWD/$out/parity_margins.jsonl
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_gpu_parity.py tests/test_compute_rsa.py -m gpu > $out/parity.log 2>&1 || { tail -40 $out/parity.log; exit 1; }
tail -4 $out/parity.log
timeout -k 10 900 $T "tests/test_benchsize.py::test_cfg5_vit_bf16_rdm" -m gpu > $out/cfg5.log 2>&1 || { tail -40 $out/cfg5.log; exit 1; }
tail -4 $out/cfg5.log
cat $out/parity_margins.jsonl
