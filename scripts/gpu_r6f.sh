#!/bin/bash
# Round 6: the plan-free full Spearman rebuilt around one pass per RDM (k_part_y: midranks from
# wave scans of the group starts + (t, y) partitioned by t) -- parity tests, then the 73k
# statistics with kernel stats (previous: spearman_full 361.4 ms, rho 0.5679174344781109; now count tables + the fused sort form).
set -o pipefail
out=gpurun_out/r6f
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_distributed_spearman.py -m gpu -k "spearman_full or bootstrap_full or hip_pieces or rdm_correlation" > $out/parity.log 2>&1 || { tail -40 $out/parity.log; exit 1; }
tail -3 $out/parity.log
timeout -k 10 600 $T tests/test_benchsize.py -m gpu -k "plan_limit" > $out/plan_limit.log 2>&1 || { tail -40 $out/plan_limit.log; exit 1; }
tail -3 $out/plan_limit.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p --output-format csv -- python scripts/probe_full73k.py > $out/full73k.log 2>&1 || { tail -20 $out/full73k.log; exit 1; }
grep -v "amdgpu.ids\|rocprofv3\|output_stream\|HSA version" $out/full73k.log
python3 scripts/kstats_summary.py $out/prof/p_kernel_stats.csv 24 1 || true
rm -f $out/prof/p_kernel_trace.csv
