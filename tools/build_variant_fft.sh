#!/bin/bash
# Experiment build: cip_fft.hip recompiled with extra defines (e.g.
# -DCIP_FFT_COLBLOCK=16), linked with the normal build's other objects into
# tools/variants/libcip_hip_<name>.so (select with CIP_HIP_LIB).
# Usage: tools/build_variant_fft.sh <name> <flags...>. Needs the normal build first.
set -e
cd "$(dirname "$0")/../ska-sdp-continuum-imaging-pipeline_amd/csrc"
name=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I../../include -I. \
  "$@" -c cip_fft.hip -o build/variant_fft_$name.o
objs=$(ls build/*.o | grep -v "build/cip_fft.o" | grep -v "build/variant_")
mkdir -p ../../tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libcip_hip_$name.so \
  $objs build/variant_fft_$name.o -L/opt/rocm/lib -lhipfft -lrccl -Wl,-rpath,/opt/rocm/lib
