#!/bin/bash
# Round 6: Kendall level kernels with 1024-thread blocks (abl/kf1024.so) against the default
# 512 (73k: kendall_full 672.5 ms, split 8.6 ms, bucket 3.7 ms per level).
set -o pipefail
out=gpurun_out/r6h
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
ALT_LIB=$PWD/abl/kf1024.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof1024 -o p --output-format csv -- python scripts/probe_full73k.py > $out/full73k_1024.log 2>&1 || { tail -20 $out/full73k_1024.log; exit 1; }
grep "kendall" $out/full73k_1024.log
python3 scripts/kstats_summary.py $out/prof1024/p_kernel_stats.csv 40 1 | grep k_kf_lvl || true
rm -f $out/prof1024/p_kernel_trace.csv
