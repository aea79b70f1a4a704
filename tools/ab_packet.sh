#!/bin/bash
# A/B of the wave-coherent (packet) traversal against the per-lane kernels on the small scenes.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_pkt}
mkdir -p $O
for C in C2 C4; do
  for P in 1 0; do
    BLING_PACKET=$P timeout -k 10 300 python -u bench.py --config $C --no-cpu --steps 3 --warmup 1 > $O/${C}_pkt$P.log 2>&1
    echo "$C packet=$P $(tail -1 $O/${C}_pkt$P.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["ms_closest_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C2_prof -o prof -- python3 bench.py --no-cpu > $O/C2_prof.log 2>&1
