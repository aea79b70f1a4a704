#!/bin/bash
# Factored-candidate A/B on C2: parity tests, bench default vs nofac (alternating, twice), and
# FETCH_SIZE / WRITE_SIZE passes of both builds for the bytes per path vertex of k_shade / k_resolve.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_fac}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 240 --timeout-method thread -k "C1 or C2 or X4 or golden" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_variants.sh ${1:-ab_fac} "C2" "default nofac default nofac"
for V in default nofac; do
  VV=$V; [ "$V" = default ] && VV=
  BLING_HIP_VARIANT=$VV timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$V -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $O/pmc_fetch_$V.log 2>&1
  BLING_HIP_VARIANT=$VV timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$V -o pmc -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $O/pmc_write_$V.log 2>&1
done
echo pmc done
