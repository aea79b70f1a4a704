set -e
O=gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/s2f_gpu_tests.log 2>&1
timeout -k 10 200 python -u tools/shard_probe.py --config C5 --worlds 2048 --reps 1 > $O/s2f_c5.log 2>&1
timeout -k 10 200 python -u bench.py --config C3 --no-cpu --steps 2 --warmup 1 > $O/s2f_c3.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu > $O/s2f_c2.log 2>&1
