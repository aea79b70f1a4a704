#!/bin/bash
# Round-3 measurement session (one GPU box, no freeze step): bench lines of
# C1..C5, rocprofv3 kernel stats per config, HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate
# runs) for C2 / C3 / C4, two SQ passes (issue / LDS / VALU lane utilisation) for C2, C4 and C5, and
# the one-GPU strong-scaling model of C2 (tools/shard_probe.py).  Then
# `python tools/collect_profiles.py gpurun_out/<TAG> <round>` copies what bench.py reads to profiles/.
# Every GPU step has its own limit; the first failure ends the script.
#   bash tools/gpu/profile_round.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03p}
O=gpurun_out/$TAG
mkdir -p $O
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"
SQB="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAVES"


timeout -k 10 300 python -u bench.py --config C1 > $O/C1_bench.log 2>&1
tail -1 $O/C1_bench.log | cut -c1-160
for C in C2 C3 C4; do
  timeout -k 10 300 python -u bench.py --config $C > $O/${C}_bench.log 2>&1
  tail -1 $O/${C}_bench.log | cut -c1-160
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${C}_prof -o prof -- python3 bench.py --config $C --no-cpu > $O/${C}_prof.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${C}_pmc_fetch -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_pmc_fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${C}_pmc_write -o pmc -- python3 bench.py --config $C --no-cpu --steps 1 --warmup 0 > $O/${C}_pmc_write.log 2>&1
  echo $C pmc ok
done
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/C2_sqa -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $O/C2_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/C2_sqb -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $O/C2_sqb.log 2>&1
echo C2 sq ok
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/C4_sqa -o pmc -- python3 bench.py --config C4 --no-cpu --steps 1 --warmup 0 > $O/C4_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/C4_sqb -o pmc -- python3 bench.py --config C4 --no-cpu --steps 1 --warmup 0 > $O/C4_sqb.log 2>&1
echo C4 sq ok
C5A="--config C5 --tile-stride 1024"
timeout -k 10 300 python -u bench.py $C5A > $O/C5_bench.log 2>&1
tail -1 $O/C5_bench.log | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/C5_prof -o prof -- python3 bench.py $C5A --no-cpu > $O/C5_prof.log 2>&1
timeout -s KILL 250 rocprofv3 --pmc $SQA --output-format csv -d $O/C5_sqa -o pmc -- python3 bench.py $C5A --no-cpu --steps 1 --warmup 0 > $O/C5_sqa.log 2>&1
timeout -s KILL 250 rocprofv3 --pmc $SQB --output-format csv -d $O/C5_sqb -o pmc -- python3 bench.py $C5A --no-cpu --steps 1 --warmup 0 > $O/C5_sqb.log 2>&1
timeout -k 10 300 python -u tools/shard_probe.py --config C2 --out $O/C2_shard_probe.json > $O/shard_probe.log 2>&1
echo shard ok
echo all done
