#!/bin/bash
# SQ stall breakdown of the bench kernels (one PMC pass, 8 SQ counters).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-sq}
cd $R
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/${TAG}_pmc_sq -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 ${BENCH_ARGS} > $O/${TAG}_pmc_sq.log 2>&1
