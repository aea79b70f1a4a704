# The Mandelbulb parity tests first (job-queue march, k_march_jobs), then the GPU suite, then C5 with
# the job-queue march (default) and the per-lane k_march (variant lane), alternating.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab5; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "C5" > $O/c5_tests.log 2>&1 || { tail -30 $O/c5_tests.log; exit 1; }
tail -1 $O/c5_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
bash tools/gpu/ab_multi.sh r03ab5 "lane" "C5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5_prof -o prof -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 --tile-stride 1024 > $O/C5_prof.log 2>&1
echo done
