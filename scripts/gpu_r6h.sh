#!/bin/bash
# Round 6: Kendall level kernels with 1024-thread blocks (abl/kf1024.so) against the default
# 512 (73k: kendall_full 672.5 ms); now x keys as the y sort payload (no k_kf_xkeys gather).
set -o pipefail
out=gpurun_out/r6h
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kendall.py tests/test_gpu_parity.py -m gpu -k "kendall or full" > $out/kendall.log 2>&1 || { tail -40 $out/kendall.log; exit 1; }
tail -2 $out/kendall.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python scripts/probe_full73k.py > $out/full73k.log 2>&1 || { tail -20 $out/full73k.log; exit 1; }
grep "kendall\|spearman" $out/full73k.log
python3 scripts/kstats_summary.py $out/prof/p_kernel_stats.csv 40 1 | grep k_kf || true
rm -f $out/prof/p_kernel_trace.csv
