set -e -o pipefail
O=gpurun_out/stk
mkdir -p $O
for R in 4 8 12 16 20; do
  BLING_STACK4_LDS=$R timeout -k 10 200 python -u bench.py --config C3 --no-cpu --steps 2 --warmup 1 > $O/C3_$R.log 2>&1
  echo "C3 rows=$R $(tail -1 $O/C3_$R.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["value"], d["ms_per_step"], c["ms_closest_per_step"])')"
done
