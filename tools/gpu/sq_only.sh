#!/bin/bash
# The two SQ counter passes of one config (the counters of final_round.sh's sq()), for a quick look at
# a kernel change; summarise with tools/collect_profiles.py's sq_summary(gpurun_out/TAG, CFG).
#   bash tools/gpu/sq_only.sh TAG "C2 C4" [extra bench.py args]
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-sq}; CFGS=${2:-C2}; shift 2 || true
O=gpurun_out/$TAG
mkdir -p $O
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"
for C in $CFGS; do
  timeout -s KILL 250 rocprofv3 --pmc $SQA --output-format csv -d $O/${C}_sqa -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 "$@" > $O/${C}_sqa.log 2>&1
  timeout -s KILL 250 rocprofv3 --pmc $SQB --output-format csv -d $O/${C}_sqb -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 "$@" > $O/${C}_sqb.log 2>&1
  echo $C sq ok
done
