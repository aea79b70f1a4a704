# Closing check of the tree as committed: GPU suite, smoke(), the default bench line (with its CPU
# baseline) and a kernel-trace summary of the same command, then C4 / C5 bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03f}; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/C2_bench.json 2> $O/C2_bench.err || exit 3
tail -c 300 $O/C2_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C2_prof -o prof -- python3 bench.py --no-cpu > $O/C2_prof.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --config C4 --no-cpu --steps 1 --warmup 1 > $O/C4_bench.json 2> $O/C4_bench.err || exit 5
timeout -k 10 300 python -u bench.py --config C5 --no-cpu --steps 2 --warmup 1 --tile-stride 1024 > $O/C5_bench.json 2> $O/C5_bench.err || exit 6
python3 -c "import json; [print(c, json.load(open('$O/'+c+'_bench.json'))['value']) for c in ('C2','C4','C5')]"
