#!/bin/bash
# PC sampling of one C2 pass (rocprofv3 beta): which instructions k_shade's waves sit on.  Each
# attempt has its own limit; a timeout ends the script.
export TMPDIR=/tmp
O=gpurun_out/${1:-pcs}; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/list.txt 2>&1; echo "list rc $?"
grep -i -A12 "pc.sampl" $O/list.txt | head -40
timeout -k 10 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 1048576 -d $O/st -o pcs -- python3 bench.py --no-cpu --steps 1 --warmup 0 > $O/st.log 2>&1
rc=$?; echo "stochastic rc $rc"; tail -5 $O/st.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
ls -la $O/st 2>/dev/null | head
exit 0
