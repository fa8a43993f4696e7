#!/bin/bash
# Interleaved A/B of one environment setting: bench.py (10 timed steps after 10
# warm-up) with and without "$1", alternating 3 times; value and phases per run
# into gpurun_out/ab_env.txt. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab_env.txt
for k in 1 2 3; do
  for cfg in "" "$1"; do
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 10 \
        > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('${cfg:-default}', d['value'], d['phases_ms'])" \
        >> gpurun_out/ab_env.txt
  done
done
