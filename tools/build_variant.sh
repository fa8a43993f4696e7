#!/bin/bash
# Experiment builds of libcip_hip.so: the W = 8 scatter unit compiled with
# extra flags (e.g. -DCIP_ABLATE=1, see cip_scatter.h); output
# tools/variants/libcip_hip_<name>.so, selected at run time with CIP_HIP_LIB.
# Usage: tools/build_variant.sh <name> <flags...>. Needs the normal build first.
set -e
cd "$(dirname "$0")/../ska-sdp-continuum-imaging-pipeline_amd/csrc"
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I../../include -I. \
  -DCIP_SCATTER_W=8 "$@" -c cip_scatter_w.hip -o build/variant_$name.o
objs="build/cip_api.o build/cip_plan.o build/cip_grid.o build/cip_tiling.o build/cip_fft.o build/cip_collective.o"
for w in 4 6 10 12 14 16; do objs="$objs build/cip_scatter_w$w.o"; done
mkdir -p ../../tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libcip_hip_$name.so \
  $objs build/variant_$name.o -L/opt/rocm/lib -lhipfft -lrccl -Wl,-rpath,/opt/rocm/lib
