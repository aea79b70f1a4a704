#!/bin/bash
# Round-4 A/B session: the default build's GPU suite, then ab_multi over per-config variant lists,
# then optional extra steps.  Every GPU step has its own limit; the first failure ends the script.
#   bash tools/gpu/r04_ab.sh TAG "C2:v1 v2" "C3 C4:v1" ...
set -e -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
  tail -1 $O/gpu_tests.log
fi
for spec in "$@"; do
  CFGS=${spec%%:*}; VARS=${spec#*:}
  bash tools/gpu/ab_multi.sh $TAG/ab "$VARS" "$CFGS"
done
if [ -n "$DIVERGENCE" ]; then
  BLING_HIP_VARIANT=dbg timeout -k 10 400 python -u tools/film_divergence.py --config C2 --stride 16 --out $O/c2_film_divergence.json > $O/c2_film_divergence.log 2>&1 || { tail -20 $O/c2_film_divergence.log; exit 7; }
  tail -20 $O/c2_film_divergence.log
fi
echo done
