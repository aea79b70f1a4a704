#!/bin/bash
# One GPU-box session of round 2: the GPU test suite (all tests, metrics in
# gpurun_out/parity_metrics.jsonl), the default bench line and a rocprofv3 kernel-trace summary of
# the same bench command.  A crash / timeout of any step ends the script (test failures do not).
#   bash tools/r02_round.sh TAG [pytest-args...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
shift
O=gpurun_out
mkdir -p $O
rm -f $O/parity_metrics.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread "$@" > $O/${TAG}_gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 $O/${TAG}_gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/${TAG}_bench.log 2>&1 || exit $?
tail -1 $O/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o prof -- python3 bench.py --no-cpu > $O/${TAG}_prof_bench.log 2>&1 || exit $?
echo done
