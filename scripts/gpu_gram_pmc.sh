#!/bin/bash
# PMC counters of the split Gram kernel (N=10k, D=43264), one rocprofv3 pass per counter group.
set -o pipefail
out=gpurun_out/${1:-gram_pmc}
mkdir -p $out
export TMPDIR=/tmp
export DS=43264
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TA_BUSY_avr"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $out/p$i -o pmc --output-format csv -- python scripts/probe_gram.py > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
echo done
