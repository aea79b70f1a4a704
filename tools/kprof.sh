#!/bin/bash
# Kernel-time breakdown of bench configs (rocprofv3 kernel trace + stats, no counters).
#   bash tools/kprof.sh TAG "C2 C3 C4"
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-kp}
mkdir -p $O
for C in $2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_prof -o prof -- python3 bench.py --config $C --no-cpu --steps 2 --warmup 1 > $O/${C}_prof.log 2>&1
  tail -1 $O/${C}_prof.log | cut -c1-200
  python3 tools/kstats.py $(find $O/${C}_prof -name "*kernel_stats.csv" | head -n 1) 3
done
