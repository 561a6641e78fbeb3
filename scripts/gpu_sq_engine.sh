#!/bin/bash
# SQ counters of the engine kernels over one 14-unit call on the bench RDMs
# (probe_engine_bench.py, REPS=1), one rocprofv3 --pmc pass per engine form.
# Usage (via gpurun): bash scripts/gpu_sq_engine.sh <tag> [forms: "tri1 tri0"]
set -o pipefail
tag=${1:-sq_engine}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp MIOPEN_FIND_MODE=FAST REPS=1 CHECK_EXACT=0
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for f in ${2:-tri1 tri0}; do
  VISREPS_ENGINE_TRI=${f#tri} timeout -s KILL 240 rocprofv3 --pmc $C -d $out/$f -o p --output-format csv \
      -- python scripts/probe_engine_bench.py > $out/$f.log 2>&1 || { echo "$f pass failed"; tail -5 $out/$f.log; exit 1; }
  python3 scripts/sq_summary.py $out/$f/p_counter_collection.csv 'k_rank|k_countA|k_join' > $out/$f.json || exit 1
  rm -f $out/$f/p_counter_collection.csv
  echo "== $f"; python3 -c "
import json,sys
d=json.load(open('$out/$f.json'))
for k,e in d.items(): print(k, e['dispatches'], e['avg_us'], 'clk', e.get('clock_ghz'), 'valu', e.get('SQ_ACTIVE_INST_VALU/wave_cycles'), 'sca', e.get('SQ_ACTIVE_INST_SCA/wave_cycles'), 'vmem', e.get('SQ_ACTIVE_INST_VMEM/wave_cycles'), 'wait_inst', e.get('SQ_WAIT_INST_ANY/wave_cycles'), 'wait_any', e.get('SQ_WAIT_ANY/wave_cycles'))
"
done
