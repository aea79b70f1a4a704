#!/bin/bash
# One GPU-box session: GPU parity tests, the default bench line, a rocprofv3 kernel-trace summary of
# the same bench command, and two PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) for the
# per-launch HBM traffic of k_trace_closest.  Every GPU step has its own time limit; the first
# failure ends the script.
#   bash tools/gpu_round.sh TAG [skip-tests]
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-run}
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1
fi
timeout -k 10 300 python -u bench.py > $O/${TAG}_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o prof -- python3 bench.py --no-cpu > $O/${TAG}_prof_bench.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_pmc_fetch -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $O/${TAG}_pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_pmc_write -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $O/${TAG}_pmc_write.log 2>&1
tail -1 $O/${TAG}_bench.log
