#!/bin/bash
# A/B of experiment builds (make variant) on the default bench: bash tools/variant_round.sh TAG v1 v2 ...
# ("main" = libbling_hip.so).  GPU parity tests run first on the main build.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=$1; shift
cd $R
if [ -z "$SKIP_TESTS" ]; then timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1; fi
i=0
for v in "$@"; do
  i=$((i+1))
  if [ "$v" = main ]; then unset BLING_HIP_VARIANT; else export BLING_HIP_VARIANT=$v; fi
  timeout -k 10 200 python -u bench.py --no-cpu --steps 4 > $O/${TAG}_bench_${i}_$v.log 2>&1
done
