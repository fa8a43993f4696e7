#!/bin/bash
# Experiment builds of libcip_hip.so: the W = 8 scatter unit compiled with
# extra flags (e.g. -DCIP_ABLATE=1, see cip_scatter.h); output
# tools/variants/libcip_hip_<name>.so, selected at run time with CIP_HIP_LIB.
# Usage: [WV=<support>] tools/build_variant.sh <name> <flags...> (WV: the
# scatter unit to replace, default 8). Needs the normal build first.
set -e
cd "$(dirname "$0")/../ska-sdp-continuum-imaging-pipeline_amd/csrc"
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I../../include -I. \
  -DCIP_SCATTER_W=${WV:-8} "$@" -c cip_scatter_w.hip -o build/variant_$name.o
# every object of the normal build except the W = 8 scatter unit (and other variants)
objs=$(ls build/*.o | grep -v "build/cip_scatter_w${WV:-8}.o" | grep -v "build/variant_")
mkdir -p ../../tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libcip_hip_$name.so \
  $objs build/variant_$name.o -L/opt/rocm/lib -lhipfft -lrccl -Wl,-rpath,/opt/rocm/lib
