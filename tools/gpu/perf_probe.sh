# Kernel-time breakdown (rocprofv3 kernel trace, no counters) of the C4 / C3 / C2 benches.
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
prof c3 --config C3 --steps 1 --warmup 1 || exit 13
prof c2 --config C2 --steps 2 --warmup 1 || exit 14
echo done
