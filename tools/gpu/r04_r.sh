set -e -o pipefail
bash tools/gpu/r04_profile2.sh r04q
SKIP_TESTS=1 PARITY="mj2" PARITY_K="full_config and C5 or film_parity_config and C5" bash tools/gpu/r04_ab.sh r04r "C5:mj2 mj2w5"
