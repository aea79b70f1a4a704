# Kernel-time breakdown (rocprofv3 kernel trace, no counters) of C3 / C4 / C5 and two A/Bs:
# binary32 ocml transcendentals (variant cr32, parity off) and a smaller C4 wave.
#   bash tools/gpu/perf_probe.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-perf}
mkdir -p $OUT
prof() {   # name, bench args...
  local N=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${N}_prof -o prof -- python3 bench.py --no-cpu "$@" > $OUT/${N}_prof.log 2>&1 || return 1
  python3 tools/kstats.py $(find $OUT/${N}_prof -name "*kernel_stats.csv" | head -n 1) 1 > $OUT/${N}_kstats.txt
}
prof c4 --config C4 --steps 1 --warmup 1 || exit 11
prof c5 --config C5 --steps 1 --warmup 1 --tile-stride 1024 || exit 12
prof c3 --config C3 --steps 1 --warmup 1 || exit 13
BLING_HIP_VARIANT=cr32 timeout -k 10 300 python3 bench.py --config C4 --no-cpu --steps 1 --warmup 1 > $OUT/c4_cr32.json 2>&1 || exit 21
BLING_HIP_VARIANT=cr32 timeout -k 10 300 python3 bench.py --config C5 --no-cpu --steps 1 --warmup 1 --tile-stride 1024 > $OUT/c5_cr32.json 2>&1 || exit 22
BLING_HIP_VARIANT=cr32 timeout -k 10 300 python3 bench.py --config C2 --no-cpu --steps 5 --warmup 2 > $OUT/c2_cr32.json 2>&1 || exit 23
timeout -k 10 300 python3 bench.py --config C4 --no-cpu --steps 1 --warmup 1 --chunk 70000000 > $OUT/c4_chunk70m.json 2>&1 || exit 24
echo done
