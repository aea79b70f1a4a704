#!/bin/bash
# Closing measurement session of a round on the final tree, in two parts (each fits one gpurun call):
#   part 1: the GPU suite, smoke, the shading kernel's counted stream bytes of C1..C4
#           (BLING_HIP_VARIANT=streams, copied into profiles/ on the box so the bench lines read them),
#           then C2 and C3: bench line, kernel trace, FETCH_SIZE and WRITE_SIZE passes, SQ passes of C2
#   part 2: the same for C4 (stream bytes again first: part 2 runs on a fresh box), the C5 and C1
#           bench lines with a C5 kernel trace, SQ passes of C4, C3 and C5, the one-GPU shard model
# Then `python tools/collect_profiles.py gpurun_out/<TAG> <ROUND>` copies the results to profiles/.
# Every GPU step has its own limit; the first failure ends the script.
#   bash tools/gpu/final_round.sh TAG ROUND 1|2
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05z}; ROUND=${2:-r05}; PART=${3:-1}
O=gpurun_out/$TAG
mkdir -p $O profiles
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"

streams() {
  local C=$1 c=$(echo $1 | tr 'A-Z' 'a-z')
  BLING_HIP_VARIANT=streams timeout -k 10 200 python -u tools/stream_bytes.py --config $C --out $O/${C}_streams.json > $O/${C}_streams.log 2>&1
  tail -1 $O/${C}_streams.log
  cp $O/${C}_streams.json profiles/${ROUND}_${c}_shade_streams.json
}
measure() {
  local C=$1
  timeout -k 10 300 python -u bench.py --config $C > $O/${C}_bench.log 2>&1
  tail -1 $O/${C}_bench.log | cut -c1-160
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_prof -o prof -- python3 bench.py --config $C --no-cpu > $O/${C}_prof.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${C}_pmc_fetch -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_pmc_fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${C}_pmc_write -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_pmc_write.log 2>&1
}
sq() {
  local C=$1; shift
  timeout -s KILL 250 rocprofv3 --pmc $SQA --output-format csv -d $O/${C}_sqa -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 "$@" > $O/${C}_sqa.log 2>&1
  timeout -s KILL 250 rocprofv3 --pmc $SQB --output-format csv -d $O/${C}_sqb -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 "$@" > $O/${C}_sqb.log 2>&1
  echo $C sq ok
}

if [ "$PART" = 1 ]; then
  rm -f gpurun_out/parity_metrics.jsonl
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
  tail -1 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
  tail -1 $O/smoke.log
  for C in C1 C2 C3 C4; do streams $C; done
  for C in C2 C3; do measure $C; done
  sq C2
else
  streams C4
  measure C4
  C5A="--tile-stride 1024"
  timeout -k 10 300 python -u bench.py --config C5 $C5A > $O/C5_bench.log 2>&1
  tail -1 $O/C5_bench.log | cut -c1-160
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5_prof -o prof -- python3 bench.py --config C5 $C5A --no-cpu > $O/C5_prof.log 2>&1
  timeout -k 10 300 python -u bench.py --config C1 > $O/C1_bench.log 2>&1
  tail -1 $O/C1_bench.log | cut -c1-160
  sq C4
  sq C3
  sq C5 $C5A
  timeout -k 10 300 python -u tools/shard_probe.py --config C2 --out $O/C2_shard_probe.json > $O/shard_probe.log 2>&1
  echo shard ok
fi
echo all done
