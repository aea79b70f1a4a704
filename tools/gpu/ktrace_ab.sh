#!/bin/bash
# Kernel-trace summaries (rocprofv3 --kernel-trace --stats) of one config under several environment
# settings, for per-kernel A/B times: gpurun_out/TAG/<CFG>_<i>/prof_kernel_stats.csv, one per setting.
#   bash tools/gpu/ktrace_ab.sh TAG CFG "NAME=V NAME=V ..."   ("-" = the default environment)
set -e -o pipefail
export TMPDIR=/tmp
TAG=$1; C=$2; SETS=${3:--}
O=gpurun_out/$TAG; mkdir -p $O
i=0
for E in $SETS; do
  if [ "$E" = "-" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_$i -o prof -- python3 bench.py --config $C --no-cpu --steps 2 --warmup 1 > $O/${C}_$i.log 2>&1
  else
    export "$E"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_$i -o prof -- python3 bench.py --config $C --no-cpu --steps 2 --warmup 1 > $O/${C}_$i.log 2>&1
    unset "${E%%=*}"
  fi
  echo "$C $i $E ok"
  i=$((i+1))
done
