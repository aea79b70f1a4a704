#!/bin/bash
# One GPU session: the GPU parity suite, then an A/B of the default build against an experiment
# build (libbling_hip_<V>.so, BLING_HIP_VARIANT) on the bench configs, alternating so box drift hits
# both, then a rocprofv3 kernel-trace summary of the default build on C2.  Every GPU step has its
# own limit; the first failure ends the script.
#   bash tools/gpu/ab_round.sh TAG VARIANT [configs...]
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-ab}; V=${2:-base}; shift 2 || true
CFGS=${*:-C2 C3 C4}
O=gpurun_out/$TAG
mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
for C in $CFGS; do
  ST=3; [ "$C" = "C4" ] && ST=1; [ "$C" = "C3" ] && ST=2
  for R in 1 2; do
    BLING_HIP_VARIANT=$V timeout -k 10 200 python -u bench.py --config $C --no-cpu --steps $ST --warmup 1 > $O/${C}_${V}_$R.json 2> $O/${C}_${V}_$R.err
    timeout -k 10 200 python -u bench.py --config $C --no-cpu --steps $ST --warmup 1 > $O/${C}_new_$R.json 2> $O/${C}_new_$R.err
    python3 -c "import json,sys; a=json.load(open('$O/${C}_${V}_$R.json')); b=json.load(open('$O/${C}_new_$R.json')); print('$C', '$V', a['value'], 'new', b['value'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C2_prof -o prof -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $O/C2_prof.log 2>&1
echo done
