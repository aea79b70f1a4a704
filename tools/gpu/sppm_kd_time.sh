#!/bin/bash
# k_sppm_kd's share of an SPPM pass: kernel traces of three passes of X13q (X13 with the
# golden's overrides, tests/golden/make_golden.py) and of the
# 480x480, 2 M-photon cornell pass (X5).
#   bash tools/gpu/sppm_kd_time.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-sppm_kd_time}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x13q -o prof -- python3 tools/sppm_probe.py --config X13 --over "image=128,96;sppm=200000,6,0.8,0.1;sppm_threads=4" --passes 3 > $O/x13q.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x5 -o prof -- python3 tools/sppm_probe.py --config X5 --over "image=480,480" --photons 2000000 --passes 3 > $O/x5.log 2>&1
echo sppm kd timing done
