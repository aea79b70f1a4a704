#!/bin/bash
# Two SQ counter passes (issue / wait / VALU / LDS / scratch) over one pass of a bench config.
#   bash tools/sq_cfg.sh TAG C4 [extra bench args]
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
C=$2
shift 2
mkdir -p $O
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/${C}_sqa -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 "$@" > $O/${C}_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/${C}_sqb -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 "$@" > $O/${C}_sqb.log 2>&1
echo "$C sq ok"
