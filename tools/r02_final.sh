#!/bin/bash
# Round-2 closing session, part 1 (one GPU box): the GPU test suite (parity metrics), the C1 bench
# line, then tools/r02_profile.sh (frozen work, C2..C5 bench lines, kernel stats, HBM PMC passes,
# SQ passes of C2 and C5).  Every GPU step has its own limit; the first failure ends the script.
#   bash tools/r02_final.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02f}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --config C1 > $O/C1_bench.log 2>&1
tail -1 $O/C1_bench.log | cut -c1-120
bash tools/r02_profile.sh $TAG
