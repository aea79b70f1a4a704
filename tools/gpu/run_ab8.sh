# GPU suite (cr_math specials written out, no huge-argument calls in the angle-only profiles), then
# A/B: default vs hb (huge-argument calls kept) on C2-C5, and the march slot count (s64 / s96) on C5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ab8; mkdir -p $O
rm -f gpurun_out/parity_metrics.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
cp gpurun_out/parity_metrics.jsonl $O/parity_metrics.jsonl
tail -1 $O/gpu_tests.log
bash tools/gpu/ab_multi.sh r03ab8 "hb" "C2 C3 C4" && bash tools/gpu/ab_multi.sh r03ab8 "hb s64 s96" "C5"
