#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/sweep.txt
for cv in 32768 16384 8192 4096; do
  CIP_CHUNK_VIS=$cv timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 10 > gpurun_out/cv_$cv.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/cv_$cv.json')); print('cv', $cv, d['phases_ms'])" >> gpurun_out/sweep.txt
done
