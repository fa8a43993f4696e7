#!/bin/bash
# Kernel-trace stats per library build: tools/gpu_kstats.sh <lib.so|default>...
# -> gpurun_out/ks_<name>/ (rocprofv3 --stats) and gpurun_out/kstats.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/kstats.txt
for lib in "$@"; do
  name=$(basename $lib .so); name=${name#libcip_hip_}
  if [ "$lib" = default ]; then unset CIP_HIP_LIB; else export CIP_HIP_LIB=$PWD/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/ks_$name -o ks --output-format csv \
    -- python3 bench.py --steps ${STEPS:-5} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:---sync} > gpurun_out/ks_$name.json 2> gpurun_out/ks_$name.err || exit 1
  python3 tools/kstats.py $name gpurun_out/ks_$name >> gpurun_out/kstats.txt || exit 1
done
