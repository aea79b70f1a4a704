#!/bin/bash
# C5 closest-kernel SQ passes (issue / VALU lane utilisation) on the bounded bench sample.
#   bash tools/c5_sq.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-c5sq}
mkdir -p $O
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"
C5A="--config C5 --tile-stride 1024"
timeout -s KILL 250 rocprofv3 --pmc $SQA --output-format csv -d $O/C5_sqa -o pmc -- python3 bench.py $C5A --no-cpu --steps 1 --warmup 0 > $O/C5_sqa.log 2>&1
timeout -s KILL 250 rocprofv3 --pmc $SQB --output-format csv -d $O/C5_sqb -o pmc -- python3 bench.py $C5A --no-cpu --steps 1 --warmup 0 > $O/C5_sqb.log 2>&1
echo c5 sq ok
