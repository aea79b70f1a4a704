#!/bin/bash
# SPPM X13q device vs oracle per pass (tools/sppm_hp_compare.py) with and without the kd-root test
# (BLING_HIP_VARIANT=nokdfull: make variant V=nokdfull DEFS=-DBLING_KD_ROOT=0), at X13q's round-5
# radius (0.5) and its round-6 radius (0.8): does the reference's root-box test explain the pair
# differences?  Each step has its own limit; the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-sppmkd}; mkdir -p $O
for R in 0.5 0.8; do
  OV="image=128,96;sppm=200000,6,$R,0.1;sppm_threads=4"
  timeout -k 10 300 python -u tools/sppm_hp_compare.py --over "$OV" > $O/kd_r$R.jsonl 2> $O/kd_r$R.err
  BLING_HIP_VARIANT=nokdfull timeout -k 10 300 python -u tools/sppm_hp_compare.py --over "$OV" > $O/nokd_r$R.jsonl 2> $O/nokd_r$R.err
  echo "radius $R done"
done
