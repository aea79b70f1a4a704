#!/bin/bash
# Experiment build for A/B runs: libbling_hip_<V>.so from the default objects (build/core) with
# some profile units recompiled under their own -D knobs (BLING_HIP_VARIANT=<V> loads it).
#   bash tools/build_mix.sh V "prof_0:-DBLING_BASE_WAVES=4" "prof_2:-DBLING_SKY_WAVES=2" ...
set -e
V=$1; shift
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-gpu-rdc -Wno-unused-result -munsafe-fp-atomics"
D=build/core_$V
rm -rf $D && mkdir -p $D && cp build/core/*.o $D/
pids=()
for spec in "$@"; do
  unit=${spec%%:*}; defs=${spec#*:}
  $HIPCC $FLAGS $defs -c -o $D/$unit.hip.o bling_amd/csrc/core/$unit.hip 2> $D/$unit.log &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
$HIPCC $FLAGS -shared -o bling_amd/_lib/libbling_hip_$V.so $D/*.o
echo built bling_amd/_lib/libbling_hip_$V.so
