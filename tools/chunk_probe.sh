set -e
O=gpurun_out
for ch in 67108864 134217728 0; do
timeout -k 10 200 python -u bench.py --config C3 --no-cpu --steps 1 --warmup 1 --chunk $ch > $O/s2e_c3_$ch.log 2>&1
done
timeout -k 10 200 python -u bench.py --no-cpu --steps 2 --warmup 1 --chunk 16777216 > $O/s2e_c2_16M.log 2>&1
