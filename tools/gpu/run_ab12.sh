# GPU parity suite on the Blinn-power-sharing build (bl), then the A/B default vs bl on C3 and C4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab12; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
BLING_HIP_VARIANT=bl timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
bash tools/gpu/ab_multi.sh r03ab12 "bl" "C3 C4 C2"
