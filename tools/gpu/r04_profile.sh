#!/bin/bash
# Round-4 measurement session: per config (default C2 C3 C4) the bench line, a rocprofv3 kernel-trace
# summary, the FETCH_SIZE and WRITE_SIZE passes (separate runs) and the shading kernel's counted
# stream bytes (BLING_HIP_VARIANT=streams, tools/stream_bytes.py); SQ passes for C2.  Then
# `python tools/collect_profiles.py gpurun_out/<TAG> <round>` copies what bench.py reads to profiles/.
# Every GPU step has its own limit; the first failure ends the script.
#   bash tools/gpu/r04_profile.sh TAG "C2 C3 C4" [sq-configs]
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04p}; CFGS=${2:-C2 C3 C4}; SQC=${3:-C2}
O=gpurun_out/$TAG
mkdir -p $O
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"
for C in $CFGS; do
  timeout -k 10 300 python -u bench.py --config $C > $O/${C}_bench.log 2>&1
  tail -1 $O/${C}_bench.log | cut -c1-160
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_prof -o prof -- python3 bench.py --config $C --no-cpu > $O/${C}_prof.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${C}_pmc_fetch -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_pmc_fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${C}_pmc_write -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_pmc_write.log 2>&1
  BLING_HIP_VARIANT=streams timeout -k 10 200 python -u tools/stream_bytes.py --config $C --out $O/${C}_streams.json > $O/${C}_streams.log 2>&1
  tail -1 $O/${C}_streams.log
done
for C in $SQC; do
  timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/${C}_sqa -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_sqa.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/${C}_sqb -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_sqb.log 2>&1
  echo $C sq ok
done
echo all done
