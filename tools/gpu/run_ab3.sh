# GPU parity suite on the default build, the C5 / X3 fractal parity tests on the deferred-march build
# (md), then the A/B of default / ns (no shape records in LDS) / md on C2, C3, C5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab3; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
BLING_HIP_VARIANT=md timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "C5 or X3" > $O/md_tests.log 2>&1 || { tail -30 $O/md_tests.log; exit 1; }
tail -1 $O/md_tests.log
bash tools/gpu/ab_multi.sh r03ab3 "ns md" "C2 C3 C5"
