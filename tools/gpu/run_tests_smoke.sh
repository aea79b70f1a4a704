# GPU suite and smoke() on the default build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03t}; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu > $O/C2_bench.json 2> $O/C2_bench.err || exit 3
python3 -c "import json; print('C2', json.load(open('$O/C2_bench.json'))['value'])"
