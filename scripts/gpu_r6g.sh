#!/bin/bash
# Round 6: Kendall level kernels staged through LDS (coalesced loads / stores) -- Kendall tests,
# then the 73k plan-free statistics with kernel stats (previous: kendall_full 906 ms, spearman_full 164 ms, tau
# 0.3986042363486459; level split 17.0 ms, bucket 5.2 ms per level; LDS-staged tiles: split 18.3, bucket 3.3).
set -o pipefail
out=gpurun_out/r6g
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_kendall.py tests/test_gpu_parity.py tests/test_distributed_spearman.py -m gpu -k "kendall or full or hip_pieces" > $out/kendall.log 2>&1 || { tail -40 $out/kendall.log; exit 1; }
tail -3 $out/kendall.log
timeout -k 10 300 $T tests/test_benchsize.py -m gpu -k "plan_limit" > $out/plan_limit.log 2>&1 || { tail -40 $out/plan_limit.log; exit 1; }
tail -2 $out/plan_limit.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python scripts/probe_full73k.py > $out/full73k.log 2>&1 || { tail -20 $out/full73k.log; exit 1; }
grep -v "amdgpu.ids\|rocprofv3\|output_stream\|HSA version\|simple_timer\|tool.cpp" $out/full73k.log
python3 scripts/kstats_summary.py $out/prof/p_kernel_stats.csv 24 1 || true
rm -f $out/prof/p_kernel_trace.csv
# A/B: the level kernels with 256-thread blocks (abl/kf256.so) against the default 512
ALT_LIB=$PWD/abl/kf256.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof256 -o p --output-format csv -- python scripts/probe_full73k.py > $out/full73k_256.log 2>&1 || { tail -20 $out/full73k_256.log; exit 1; }
grep "kendall" $out/full73k_256.log
python3 scripts/kstats_summary.py $out/prof256/p_kernel_stats.csv 40 1 | grep k_kf_lvl || true
rm -f $out/prof256/p_kernel_trace.csv
