#!/bin/bash
# A/B of the default build against experiment builds (libbling_hip_<V>.so, BLING_HIP_VARIANT) on
# one box: per config, two rounds, each round runs every build once in turn so drift hits all of
# them alike.  Prints one line per round: config, then per build Mrays/s / the dominant kernel's ms per
# pass / the closest-hit queries' ms per step.
#   bash tools/gpu/ab_multi.sh TAG "V1 V2 ..." "C2 C4 ..."   (a V of the form NAME=VALUE runs the default
#   build with that environment variable set)
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-abm}; VARS=${2:-}; CFGS=${3:-C2}
O=gpurun_out/$TAG
mkdir -p $O
for C in $CFGS; do
  ST=3; [ "$C" = "C4" ] && ST=1; [ "$C" = "C3" ] && ST=2
  EXTRA=""; [ "$C" = "C5" ] && EXTRA="--tile-stride 1024" && ST=2
  for R in 1 2; do
    line="$C r$R"
    for V in default $VARS; do
      if [ "$V" = "default" ]; then
        timeout -k 10 240 python -u bench.py --config $C --no-cpu --steps $ST --warmup 1 $EXTRA > $O/${C}_${V}_$R.json 2> $O/${C}_${V}_$R.err
      elif [[ "$V" == *=* ]]; then    # NAME=VALUE: the default build with that environment variable
        env "$V" timeout -k 10 240 python -u bench.py --config $C --no-cpu --steps $ST --warmup 1 $EXTRA > $O/${C}_${V}_$R.json 2> $O/${C}_${V}_$R.err
      else
        BLING_HIP_VARIANT=$V timeout -k 10 240 python -u bench.py --config $C --no-cpu --steps $ST --warmup 1 $EXTRA > $O/${C}_${V}_$R.json 2> $O/${C}_${V}_$R.err
      fi
      v=$(python3 -c "import json; d=json.load(open('$O/${C}_${V}_$R.json')); r=d['roofline']; print('%s/sh%.1f/cl%.1f' % (d['value'], r.get('ms_per_pass', 0), d['config'].get('ms_closest_per_step', 0)))")
      line="$line $V=$v"
    done
    echo "$line" | tee -a $O/summary.txt
  done
done
echo done
