#!/bin/bash
# Reference-call (secondary.reference_call) phase times per variant given as
# args, interleaved ${REPS:-2} times, into gpurun_out/ab_refcall.txt. A
# variant is "default" (the in-tree build), a library path (CIP_HIP_LIB) or
# "env:NAME=VALUE" (an environment switch on the in-tree build).
mkdir -p gpurun_out; rm -f gpurun_out/ab_refcall.txt
for rep in $(seq ${REPS:-2}); do
  for v in "$@"; do
    (
      case "$v" in
        default) ;;
        env:*) export "${v#env:}" ;;
        *) export CIP_HIP_LIB=$v ;;
      esac
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-strong-secondary --no-max-err --steps 10 --warmup 5 \
          > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
      python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); r=d['secondary']['reference_call']; print('$v', d['value'], d['phases_ms'], r['value'], r['phases_ms_sync'])" \
          >> gpurun_out/ab_refcall.txt
    ) || exit 1
  done
done
