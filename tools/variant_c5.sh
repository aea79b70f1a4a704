#!/bin/bash
# A/B of experiment builds on a bounded C5 sample (every 1024th tile): bash tools/variant_c5.sh TAG v1 v2 ...
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=$1; shift
cd $R
for v in "$@"; do
  if [ "$v" = main ]; then unset BLING_HIP_VARIANT; else export BLING_HIP_VARIANT=$v; fi
  timeout -k 10 200 python -u bench.py --config C5 --no-cpu --steps 1 --warmup 0 --tile-stride 1024 > $O/${TAG}_c5_$v.log 2>&1
done
