#!/bin/bash
# Round-4: C5 SQ passes on the closing tree (the march instruction mix), collected on the box so the
# final C5 bench line cites them; then `python tools/collect_profiles.py gpurun_out/r04c5 r04` here.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c5
mkdir -p $O
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"
A="--config C5 --tile-stride 1024"
timeout -k 10 300 python -u bench.py $A --no-cpu > $O/C5_bench.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/C5_sqa -o pmc -- python3 bench.py $A --no-cpu --steps 1 --warmup 0 > $O/C5_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/C5_sqb -o pmc -- python3 bench.py $A --no-cpu --steps 1 --warmup 0 > $O/C5_sqb.log 2>&1
python3 tools/collect_profiles.py $O r04
timeout -k 10 300 python -u bench.py $A > $O/C5_bench2.log 2>&1
tail -1 $O/C5_bench2.log | cut -c1-160
