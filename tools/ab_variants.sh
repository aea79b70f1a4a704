#!/bin/bash
# A/B of core build variants (make variant V=name DEFS=...) on bench configs.
#   bash tools/ab_variants.sh TAG "C4 C2" "default sw2 sw3"
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}
mkdir -p $O
for C in $2; do
  for V in $3; do
    VV=$V; [ "$V" = default ] && VV=
    BLING_HIP_VARIANT=$VV timeout -k 10 300 python -u bench.py --config $C --no-cpu --steps 3 --warmup 1 $4 > $O/${C}_$V.log 2>&1
    echo "$C $V $(tail -1 $O/${C}_$V.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["ms_closest_per_step"], c["ms_bounce_per_step"])')"
  done
done
