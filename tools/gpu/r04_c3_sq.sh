#!/bin/bash
# Round-4: SQ passes of C3 on the closing tree (issue / wait / lane utilisation per kernel), for the
# next round's C3 work; `python tools/collect_profiles.py gpurun_out/r04c3 r04` copies them here.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c3
mkdir -p $O
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/C3_sqa -o pmc -- python3 bench.py --config C3 --no-cpu --steps 1 --warmup 0 > $O/C3_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/C3_sqb -o pmc -- python3 bench.py --config C3 --no-cpu --steps 1 --warmup 0 > $O/C3_sqb.log 2>&1
echo C3 sq ok
