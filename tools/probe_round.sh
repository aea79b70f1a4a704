#!/bin/bash
# Kernel-time summaries of the non-headline configs on one GPU (bounded tile shards).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-probe}
cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_c3 -o prof -- python3 tools/shard_probe.py --config C3 --worlds 8 --reps 1 > $O/${TAG}_c3.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_c5 -o prof -- python3 tools/shard_probe.py --config C5 --worlds 2048 --reps 1 > $O/${TAG}_c5.log 2>&1
