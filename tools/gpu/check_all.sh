# One GPU session: first-divergence records (debug build), the GPU parity suite, and the benches.
# Usage (on the box): bash tools/gpu/check_all.sh <tag>
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
rm -f gpurun_out/parity_metrics.jsonl
BLING_HIP_VARIANT=dbg timeout -k 10 300 python -u tools/vertex_divergence.py --config C5 --out $OUT/c5_divergence.json > $OUT/div_c5.log 2>&1 || exit 11
BLING_HIP_VARIANT=dbg timeout -k 10 200 python -u tools/vertex_divergence.py --config C4 --out $OUT/c4_divergence.json > $OUT/div_c4.log 2>&1 || exit 12
BLING_HIP_VARIANT=dbg timeout -k 10 200 python -u tools/vertex_divergence.py --config C2 --out $OUT/c2_divergence.json > $OUT/div_c2.log 2>&1 || exit 13
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?
cp gpurun_out/parity_metrics.jsonl $OUT/parity_metrics.jsonl 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit 21
timeout -k 10 300 python -u bench.py --config C4 --steps 2 --warmup 1 --no-cpu > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 22
timeout -k 10 300 python -u bench.py --config C5 --steps 2 --warmup 1 --no-cpu --tile-stride 1024 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 23
timeout -k 10 300 python -u bench.py --config C3 --steps 2 --warmup 1 --no-cpu > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 24
timeout -k 10 300 python -u tools/shard_probe.py --config C2 --out $OUT/c2_shard_probe.json > $OUT/shard_probe.log 2>&1 || exit 25
echo "tests rc=$rc"
