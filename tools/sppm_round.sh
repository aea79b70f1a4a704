#!/bin/bash
# SPPM GPU session: parity tests, probes (parity figures + timing, PNGs) and a kernel-trace profile.
set -e
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=${1:-sppm}
timeout -k 10 300 python -u -m pytest tests/test_sppm.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/${TAG}_tests.log 2>&1
timeout -k 10 200 python -u tools/sppm_probe.py --config X5 --passes 4 --oracle-passes 1 > $O/${TAG}_x5.log 2>&1
timeout -k 10 200 python -u tools/sppm_probe.py --config X5 --photons 2000000 --passes 4 --oracle-passes 1 --png $O/${TAG}_x5_2M.png > $O/${TAG}_x5_2M.log 2>&1
timeout -k 10 200 python -u tools/sppm_probe.py --config X6 --photons 2000000 --passes 2 --oracle-passes 1 --png $O/${TAG}_x6_2M.png > $O/${TAG}_x6_2M.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o prof -- python3 tools/sppm_probe.py --config X5 --photons 2000000 --passes 3 > $O/${TAG}_prof.log 2>&1
tail -n 3 $O/${TAG}_tests.log; cut -c1-420 $O/${TAG}_x5*.log $O/${TAG}_x6_2M.log
