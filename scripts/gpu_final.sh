#!/bin/bash
# Round-end check on the GPU box: full parity suite + smoke, bench line, rocprofv3 kernel
# stats of the bench, and one PMC pass (MFMA busy) over the N=10k Gram probe.
set -o pipefail
tag=${1:-final}
out=gpurun_out/$tag
bash scripts/gpu_check.sh $tag || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
DS=43264 timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d $out/pmc -o pmc --output-format csv -- python scripts/probe_gram.py > $out/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $out/pmc.log; exit 1; }
echo done
