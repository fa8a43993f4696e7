#!/bin/bash
# Bench per environment setting with phases: tools/ab_env_phases.sh VAR val1 val2 ... ("-" = unset);
# two interleaved rounds -> gpurun_out/ab_phases.txt
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab_phases.txt
var=$1; shift
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = "-" ]; then unset $var; else export $var=$v; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-max-err --steps 20 --warmup 10 ${BENCH_ARGS} \
        > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$var=$v', d['value'], d['ms_per_step'], d['value_sync'], d['ms_per_step_sync'], d['phases_ms'])" \
        >> gpurun_out/ab_phases.txt
  done
done
