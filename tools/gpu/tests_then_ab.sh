#!/bin/bash
# The GPU parity suite, then ab_multi.sh.  Every GPU step has its own limit; the first failure ends it.
#   bash tools/gpu/tests_then_ab.sh TAG "V1 V2 ..." "C2 ..."
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
bash tools/gpu/ab_multi.sh "$1" "$2" "$3"
