#!/bin/bash
# One PMC counter (default FETCH_SIZE) per library build, synchronous bench steps:
# tools/gpu_pmc_libs.sh <lib.so|default>... -> gpurun_out/pmcl_<name>/
set -o pipefail
export TMPDIR=/tmp
CNT=${CNT:-FETCH_SIZE}
mkdir -p gpurun_out
for lib in "$@"; do
  name=$(basename $lib .so); name=${name#libcip_hip_}
  if [ "$lib" = default ]; then unset CIP_HIP_LIB; else export CIP_HIP_LIB=$PWD/$lib; fi
  timeout -k 10 300 rocprofv3 --pmc $CNT -d $PWD/gpurun_out/pmcl_$name -o pmcl --output-format csv \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sync > gpurun_out/pmcl_$name.json 2> gpurun_out/pmcl_$name.err || exit 1
done
