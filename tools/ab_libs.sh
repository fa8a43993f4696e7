#!/bin/bash
# Short bench per library build (CIP_HIP_LIB) given as args; value and phase
# times per variant into gpurun_out/ab_libs.txt. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab_libs.txt
for lib in "$@"; do
  if [ "$lib" = default ]; then unset CIP_HIP_LIB; else export CIP_HIP_LIB=$lib; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup ${WARMUP:-10} ${BENCH_ARGS} \
      > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$lib', d['value'], d['phases_ms'])" \
      >> gpurun_out/ab_libs.txt
done
