#!/bin/bash
# Experiment builds of libcip_hip.so with ONE translation unit compiled with
# extra flags: tools/build_variant_unit.sh <unit> <name> <flags...>, unit one
# of api plan grid tiling fft collective scatter_w<W>; output
# tools/variants/libcip_hip_<name>.so (select with CIP_HIP_LIB). Needs the
# normal build first (its objects are reused for the other units).
set -e
cd "$(dirname "$0")/../ska-sdp-continuum-imaging-pipeline_amd/csrc"
unit=$1; name=$2; shift 2
src=cip_$unit.hip; extra=""
case $unit in scatter_w*) src=cip_scatter_w.hip; extra="-DCIP_SCATTER_W=${unit#scatter_w}";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I../../include -I. \
  $extra "$@" -c $src -o build/variant_$name.o
objs=""
for u in api plan grid tiling fft collective strips scatter_w4 scatter_w6 scatter_w8 scatter_w10 scatter_w12 scatter_w14 scatter_w16 \
         scatter_large_w24 scatter_large_w32 scatter_large_w48 scatter_large_w64; do
  [ "$u" = "$unit" ] || objs="$objs build/cip_$u.o"
done
mkdir -p ../../tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libcip_hip_$name.so \
  $objs build/variant_$name.o -L/opt/rocm/lib -lhipfft -lrccl -Wl,-rpath,/opt/rocm/lib
