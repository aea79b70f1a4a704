set -e
O=gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/${TAG:-q}_gpu_tests.log 2>&1
timeout -k 10 200 python -u tools/shard_probe.py --config C5 --worlds 2048 --reps 1 > $O/${TAG:-q}_c5.log 2>&1
timeout -k 10 200 python -u bench.py --config C3 --no-cpu --steps 2 --warmup 1 > $O/${TAG:-q}_c3.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu > $O/${TAG:-q}_c2.log 2>&1
