#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration runs of tools/pmc_calib (separate --pmc passes).
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-calib}
mkdir -p $O
timeout -k 10 120 ./tools/pmc_calib > $O/calib_plain.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o pmc -- ./tools/pmc_calib > $O/calib_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o pmc -- ./tools/pmc_calib > $O/calib_write.log 2>&1
cat $O/calib_plain.log
