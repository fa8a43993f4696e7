#!/bin/bash
# Experiment build of the WHOLE library (every unit, per-W scatter objects
# included) with extra compile flags:
#   tools/build_variant_all.sh NAME "-DFOO=1 ..."
# output tools/variants/libcip_hip_NAME.so (select with CIP_HIP_LIB)
set -e
name=$1; defs=$2
cd "$(dirname "$0")/../ska-sdp-continuum-imaging-pipeline_amd/csrc"
B=build_$name; mkdir -p $B ../../tools/variants
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I../../include -I. $defs"
pids=""
for u in api plan grid tiling fft collective strips; do /opt/rocm/bin/hipcc $F -c cip_$u.hip -o $B/cip_$u.o & pids="$pids $!"; done
for w in 4 6 8 10 12 14 16; do /opt/rocm/bin/hipcc $F -DCIP_SCATTER_W=$w -c cip_scatter_w.hip -o $B/cip_scatter_w$w.o & pids="$pids $!"; done
for w in 24 32 48 64; do /opt/rocm/bin/hipcc $F -DCIP_LARGE_W=$w -c cip_scatter_large.hip -o $B/cip_scatter_large_w$w.o & pids="$pids $!"; done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libcip_hip_$name.so $B/*.o \
  -L/opt/rocm/lib -lhipfft -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $B
