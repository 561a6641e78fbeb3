#!/bin/bash
# SQ counters + GRBM_GUI_ACTIVE (the clock) of the wide Gram kernels on probe_gram.py
# (N = 10k, random rows): k_gram3e (default) and k_gram3p (VISREPS_GRAM_KERNEL=p), at two
# depths. One rocprofv3 --pmc pass per (kernel, depth).
set -o pipefail
out=gpurun_out/${1:-gram_pmc_e}
mkdir -p $out
export TMPDIR=/tmp REPS=2
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
for kern in e p; do
  for ds in 43264 290400; do
    VISREPS_GRAM_KERNEL=$kern DS=$ds timeout -s KILL 120 rocprofv3 --pmc $C -d $out/$kern$ds -o p --output-format csv \
        -- python scripts/probe_gram.py > $out/$kern$ds.log 2>&1 || { echo "pmc $kern $ds failed"; tail -5 $out/$kern$ds.log; exit 1; }
    python3 scripts/gram_pmc_summary.py $out/$kern$ds/p_counter_collection.csv $kern $ds
  done
done
