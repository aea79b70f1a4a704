#!/bin/bash
# SPPM treeLookup mirror on the GPU: device vs oracle per pass on scenes whose radii fall below 1
# and differ per pixel (X13 with alpha 0.1), then the SPPM GPU tests.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-sppm_kd}; mkdir -p $O
V=${2:-}
export BLING_HIP_VARIANT=$V
timeout -k 10 300 python -u tools/sppm_probe.py --config X13 --over "image=256,192;sppm=400000,6,0.5,0.1;sppm_threads=4" --passes 3 --oracle-passes 3 > $O/x13_quirk.jsonl 2> $O/x13_quirk.err
timeout -k 10 300 python -u tools/sppm_probe.py --config X6 --over "image=96,54;sppm_threads=4" --passes 3 --oracle-passes 3 > $O/x6.jsonl 2> $O/x6.err
timeout -k 10 300 python -u -m pytest tests/test_sppm.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/sppm_tests.log 2>&1 || { tail -30 $O/sppm_tests.log; exit 1; }
tail -1 $O/sppm_tests.log
cat $O/x13_quirk.jsonl
