#!/bin/bash
# SQ stall / instruction-mix breakdown of the bench kernels (one PMC pass, 8 SQ counters).
#   BENCH_ARGS="--config C5 --tile-stride 1024" bash tools/pmc_sq.sh TAG
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-sq}
cd $R
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/${TAG}_pmc_sq -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 ${BENCH_ARGS} > $O/${TAG}_pmc_sq.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAVES --output-format csv -d $O/${TAG}_pmc_valu -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 ${BENCH_ARGS} > $O/${TAG}_pmc_valu.log 2>&1
