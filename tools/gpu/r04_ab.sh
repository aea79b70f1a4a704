#!/bin/bash
# Round-4 A/B session: the default build's GPU suite, then ab_multi over per-config variant lists,
# then optional extra steps.  Every GPU step has its own limit; the first failure ends the script.
#   bash tools/gpu/r04_ab.sh TAG "C2:v1 v2" "C3 C4:v1" ...
set -e -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
  tail -1 $O/gpu_tests.log
fi
for spec in "$@"; do
  CFGS=${spec%%:*}; VARS=${spec#*:}
  bash tools/gpu/ab_multi.sh $TAG/ab "$VARS" "$CFGS"
done
if [ -n "$DIVERGENCE" ]; then
  BLING_HIP_VARIANT=dbg timeout -k 10 400 python -u tools/film_divergence.py --config C2 --stride 16 --out $O/c2_film_divergence.json > $O/c2_film_divergence.log 2>&1 || { tail -20 $O/c2_film_divergence.log; exit 7; }
  tail -20 $O/c2_film_divergence.log
fi
for V in ${PARITY:-}; do
  BLING_HIP_VARIANT=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "${PARITY_K:-trace or full_config}" > $O/parity_$V.log 2>&1 || { tail -30 $O/parity_$V.log; exit 6; }
  echo "parity $V: $(tail -1 $O/parity_$V.log)"
done
for C in ${STREAMS:-}; do
  BLING_HIP_VARIANT=streams timeout -k 10 200 python -u tools/stream_bytes.py --config $C --out $O/${C}_streams.json > $O/${C}_streams.log 2>&1 || exit 8
  tail -1 $O/${C}_streams.log
done
if [ -n "$CALIB" ]; then
  bash tools/pmc_calib.sh $TAG/calib || exit 9
fi
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"
for C in ${SQC:-}; do
  timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/${C}_sqa -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_sqa.log 2>&1 || exit 10
  timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/${C}_sqb -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_sqb.log 2>&1 || exit 11
  echo $C sq ok
done
echo done
