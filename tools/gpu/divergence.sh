set -o pipefail
export BLING_HIP_VARIANT=dbg
timeout -k 10 300 python -u tools/vertex_divergence.py --config C5 --out gpurun_out/r03_c5_divergence.json > gpurun_out/div_c5.log 2>&1 &&
timeout -k 10 200 python -u tools/vertex_divergence.py --config C4 --out gpurun_out/r03_c4_divergence.json > gpurun_out/div_c4.log 2>&1 &&
timeout -k 10 200 python -u tools/vertex_divergence.py --config C2 --out gpurun_out/r03_c2_divergence.json > gpurun_out/div_c2.log 2>&1
echo rc=$?
