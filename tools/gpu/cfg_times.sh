#!/bin/bash
# Per-config bench lines of the default build (C2, C3, C4, C5 at their bench settings, no CPU
# baseline), each under its own limit; the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-cfg}; mkdir -p $O
for C in ${2:-C3 C4 C5}; do
  ST=3; [ "$C" = "C4" ] && ST=1; [ "$C" = "C3" ] && ST=2
  EXTRA=""; [ "$C" = "C5" ] && EXTRA="--tile-stride 1024" && ST=2
  timeout -k 10 300 python -u bench.py --config $C --no-cpu --steps $ST --warmup 1 $EXTRA > $O/$C.json 2> $O/$C.err
  python3 -c "import json; d=json.load(open('$O/$C.json')); r=d['roofline']; print('$C', d['value'], r.get('kernel'), r.get('ms_per_pass'), d['config'].get('ms_closest_per_step'))" | tee -a $O/summary.txt
done
