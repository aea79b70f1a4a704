# GPU parity suite (Mandelbulb queries pre-marched by k_march), then C5 with and without the
# pre-march (BLING_PREMARCH=0), alternating, and a kernel-trace summary of C5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab4; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
for R in 1 2; do
  BLING_PREMARCH=0 timeout -k 10 240 python -u bench.py --config C5 --no-cpu --steps 2 --warmup 1 --tile-stride 1024 > $O/C5_inline_$R.json 2> $O/C5_inline_$R.err || exit 21
  timeout -k 10 240 python -u bench.py --config C5 --no-cpu --steps 2 --warmup 1 --tile-stride 1024 > $O/C5_pre_$R.json 2> $O/C5_pre_$R.err || exit 22
  python3 -c "import json; print('C5 r$R inline', json.load(open('$O/C5_inline_$R.json'))['value'], 'pre', json.load(open('$O/C5_pre_$R.json'))['value'])" | tee -a $O/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5_prof -o prof -- python3 bench.py --config C5 --no-cpu --steps 2 --warmup 1 --tile-stride 1024 > $O/C5_prof.log 2>&1
echo done
