set -e
O=gpurun_out
timeout -k 10 300 python -u tools/freeze_roofline.py C2 C3 C4 C5 > $O/s2l_freeze.log 2>&1
timeout -k 10 200 python -u bench.py --config C4 --no-cpu --steps 1 --warmup 1 > $O/s2l_c4.log 2>&1
timeout -k 10 200 python -u bench.py --config C5 --no-cpu --steps 1 --warmup 0 --tile-stride 1024 > $O/s2l_c5.log 2>&1
