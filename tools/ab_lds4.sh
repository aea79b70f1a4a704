#!/bin/bash
# A/B of the BVH4 LDS block budget (BLING_LDS4_BUDGET_KB) on C3.
set -e -o pipefail
O=gpurun_out/${1:-lds4}
mkdir -p $O
for B in 20 26 30 40 53; do
  BLING_LDS4_BUDGET_KB=$B timeout -k 10 200 python -u bench.py --config C3 --no-cpu --steps 2 --warmup 1 > $O/C3_$B.log 2>&1
  echo "C3 budget=${B}KiB $(tail -1 $O/C3_$B.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["ms_closest_per_step"])')"
done
