#!/bin/bash
# Experiment build of the whole library with extra defines:
#   tools/build_variant_full.sh NAME "-DCIP_TILE=48 ..."
# output tools/variants/libcip_hip_NAME.so (select with CIP_HIP_LIB)
set -e
name=$1; defs=$2
cd "$(dirname "$0")/../ska-sdp-continuum-imaging-pipeline_amd/csrc"
mkdir -p build_$name ../../tools/variants
for f in $(ls *.hip | sed "s/\.hip$//"); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I../../include -I. $defs \
    -c $f.hip -o build_$name/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/variants/libcip_hip_$name.so \
  build_$name/*.o -L/opt/rocm/lib -lhipfft -Wl,-rpath,/opt/rocm/lib
rm -rf build_$name
