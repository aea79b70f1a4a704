#!/bin/bash
# SPPM treeLookup mirror on the GPU: device vs oracle per pass on X13q (radii below 1 that differ
# per pixel): hit-point sets by key, pairs, radii (tools/sppm_hp_compare.py).
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-sppm_kd}; mkdir -p $O
timeout -k 10 300 python -u tools/sppm_hp_compare.py > $O/hp_compare.jsonl 2> $O/hp_compare.err
cat $O/hp_compare.jsonl
