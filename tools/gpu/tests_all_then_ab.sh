#!/bin/bash
# The whole GPU parity suite without stopping at the first failure (every test reports its metrics to
# gpurun_out/parity_metrics.jsonl), then ab_multi.sh.  Test failures (pytest exit 1) go on to the A/B;
# any other exit (time limit, crash, abort) ends the script.
#   bash tools/gpu/tests_all_then_ab.sh TAG "V1 V2 ..." "C2 ..."
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
rc=$?
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl 2>/dev/null
tail -1 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
[ -z "$2$3" ] && exit $rc
set -e
bash tools/gpu/ab_multi.sh "$1" "$2" "$3"
