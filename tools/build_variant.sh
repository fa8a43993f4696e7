#!/bin/bash
# Experiment builds of libcip_hip.so with cip_grid.hip compiled under
# -DCIP_ABLATE=N (see cip_grid.hip); output tools/variants/libcip_hip_ablN.so,
# selected at run time with CIP_HIP_LIB. Needs the normal build first.
set -e
cd "$(dirname "$0")/../ska-sdp-continuum-imaging-pipeline_amd/csrc"
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I../../include -I. \
    -DCIP_ABLATE=$n -c cip_grid.hip -o build/cip_grid_abl$n.o &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libcip_hip_abl$n.so \
    build/cip_api.o build/cip_plan.o build/cip_grid_abl$n.o build/cip_tiling.o build/cip_fft.o \
    build/cip_collective.o -L/opt/rocm/lib -lhipfft -lrccl \
    -Wl,-rpath,/opt/rocm/lib
done
