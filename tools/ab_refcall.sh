#!/bin/bash
# Reference-call (secondary.reference_call) phase times per library build
# given as args (CIP_HIP_LIB; "default" = the in-tree build), interleaved
# ${REPS:-2} times, into gpurun_out/ab_refcall.txt.
mkdir -p gpurun_out; rm -f gpurun_out/ab_refcall.txt
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset CIP_HIP_LIB; else export CIP_HIP_LIB=$lib; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-strong-secondary --no-max-err --steps 10 --warmup 5 \
        > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); r=d['secondary']['reference_call']; print('$lib', d['value'], r['value'], r['phases_ms_sync'])" \
        >> gpurun_out/ab_refcall.txt
  done
done
unset CIP_HIP_LIB
