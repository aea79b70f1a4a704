# GPU suite (material-class shading rings; depth-0 shade timed with the others), then the A/B
# default vs r1 (one ring) on C4, and a default bench line each of C2 and C3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab11; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
bash tools/gpu/ab_multi.sh r03ab11 "r1" "C4"
timeout -k 10 200 python -u bench.py --no-cpu > $O/C2_bench.json 2> $O/C2_bench.err
tail -c 400 $O/C2_bench.json
