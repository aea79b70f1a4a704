#!/bin/bash
# A/B of the BVH leaf-size cap (BLING_BVH_LEAF, upload-time) on bench configs.
#   bash tools/ab_leaf.sh TAG "C2 C3" "2 4 8"
set -e -o pipefail
O=gpurun_out/${1:-leaf}
mkdir -p $O
for C in $2; do
  for Lf in $3; do
    BLING_BVH_LEAF=$Lf timeout -k 10 200 python -u bench.py --config $C --no-cpu --steps 3 --warmup 1 > $O/${C}_$Lf.log 2>&1
    echo "$C leaf=$Lf $(tail -1 $O/${C}_$Lf.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["ms_closest_per_step"], c["ms_bounce_per_step"])')"
  done
done
