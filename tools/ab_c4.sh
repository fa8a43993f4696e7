#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab_c4.txt
for k in 1 2; do
  for cfg in "CIP_X=0" "CIP_CHUNK_VIS=8192" "CIP_CHUNK_ORDER=tile"; do
    env $cfg timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --steps 10 --warmup 5 \
        > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$cfg', d['value'], d['phases_ms'])" >> gpurun_out/ab_c4.txt
  done
done
