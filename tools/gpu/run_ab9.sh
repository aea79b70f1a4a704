# GPU suite (exact fast reciprocal in the triangle test and the traversal's ray set-up), then the
# A/B default vs div (IEEE division there) on C2, C3, C4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab9; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
bash tools/gpu/ab_multi.sh r03ab9 "div" "C2 C3 C4"
