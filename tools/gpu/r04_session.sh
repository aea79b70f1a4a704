#!/bin/bash
# Round-4 GPU session: the default build's GPU suite, smoke and C2 bench line with a kernel-trace
# summary, then an A/B of experiment builds (BLING_HIP_VARIANT) against it, and the first build's
# parity suite.  Every GPU step has its own limit; the first failure ends the script.
#   bash tools/gpu/r04_session.sh TAG "V1 V2" "C2 C4"
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04}; VARS=${2:-}; CFGS=${3:-C2}
O=gpurun_out/$TAG
mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/C2_bench.json 2> $O/C2_bench.err || exit 3
cut -c1-200 $O/C2_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C2_prof -o prof -- python3 bench.py --no-cpu > $O/C2_prof.log 2>&1 || exit 4
if [ -n "$VARS" ]; then
  bash tools/gpu/ab_multi.sh $TAG/ab "$VARS" "$CFGS"
fi
V1=${PARITY_VARIANT:-}
if [ -n "$V1" ]; then
  rm -f gpurun_out/parity_metrics.jsonl
  BLING_HIP_VARIANT=$V1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests_$V1.log 2>&1 || { tail -30 $O/gpu_tests_$V1.log; exit 5; }
  cp gpurun_out/parity_metrics.jsonl $O/parity_metrics_$V1.jsonl
  tail -1 $O/gpu_tests_$V1.log
fi
if [ -f bling_amd/_lib/libbling_hip_streams.so ]; then
  BLING_HIP_VARIANT=streams timeout -k 10 200 python -u tools/stream_bytes.py --config C2 --out $O/C2_streams.json > $O/C2_streams.log 2>&1 || exit 6
  tail -1 $O/C2_streams.log
fi
echo done
