#!/bin/bash
# Round-4 measurement session, part 2 (after the counted stream bytes of C2 / C3 are in profiles/):
# bench lines and kernel-trace summaries of C2, C3, C4 (their shade roofline now reads the counted
# bytes), C4's FETCH / WRITE passes and stream bytes, the C5 and C1 bench lines with a C5 kernel
# trace.  Every GPU step has its own limit; the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04q}
mkdir -p $O
timeout -k 10 200 python -u bench.py --config C4 --no-cpu --steps 1 --warmup 0 > /dev/null 2>&1 || true
BLING_HIP_VARIANT=streams timeout -k 10 200 python -u tools/stream_bytes.py --config C4 --out $O/C4_streams.json > $O/C4_streams.log 2>&1
tail -1 $O/C4_streams.log
mkdir -p profiles && cp $O/C4_streams.json profiles/r04_c4_shade_streams.json
for C in C2 C3 C4; do
  timeout -k 10 300 python -u bench.py --config $C > $O/${C}_bench.log 2>&1
  tail -1 $O/${C}_bench.log | cut -c1-160
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_prof -o prof -- python3 bench.py --config $C --no-cpu > $O/${C}_prof.log 2>&1
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/C4_pmc_fetch -o pmc -- python3 bench.py --config C4 --no-cpu --steps 1 --warmup 0 > $O/C4_pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/C4_pmc_write -o pmc -- python3 bench.py --config C4 --no-cpu --steps 1 --warmup 0 > $O/C4_pmc_write.log 2>&1
C5A="--config C5 --tile-stride 1024"
timeout -k 10 300 python -u bench.py $C5A > $O/C5_bench.log 2>&1
tail -1 $O/C5_bench.log | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5_prof -o prof -- python3 bench.py $C5A --no-cpu > $O/C5_prof.log 2>&1
timeout -k 10 300 python -u bench.py --config C1 > $O/C1_bench.log 2>&1
tail -1 $O/C1_bench.log | cut -c1-160
echo all done
