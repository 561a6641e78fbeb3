#!/bin/bash
# configs[4] / configs[2] legs: timed JSON, rocprofv3 kernel stats of the same command.
# Usage (via gpurun): bash scripts/gpu_legs.sh <tag>
set -o pipefail
tag=${1:-legs}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/bench_legs.py configs4 configs2 > $out/legs.jsonl 2> $out/legs.err \
    || { echo "legs failed"; tail -20 $out/legs.err; exit 1; }
cat $out/legs.jsonl | cut -c1-3000
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o legs -- \
    python -u $GRAFT_REPO_ROOT/scripts/bench_legs.py configs4 configs2 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 \
    || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $out/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats_summary.py "$f" > $out/kernel_stats.txt 2>&1 && head -25 $out/kernel_stats.txt
# SQ counters + clock of the wide Gram kernel on the configs[4] shapes (one --pmc pass)
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/$out/pmc -o p -- \
    python -u $GRAFT_REPO_ROOT/scripts/bench_legs.py configs4 > $GRAFT_REPO_ROOT/$out/pmc.log 2>&1 \
    || { echo "pmc failed"; tail -5 $GRAFT_REPO_ROOT/$out/pmc.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find $out/pmc -name "*counter_collection.csv" | head -1)
python3 scripts/gram_pmc_summary.py "$f" e 151296 > $out/gram_pmc.json && cut -c1-1500 $out/gram_pmc.json
