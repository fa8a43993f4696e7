#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.txt
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for o in 1 0; do for cv in 32768 4096; do
  CIP_SCATTER_ORDER=$o CIP_CHUNK_VIS=$cv timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_$o_$cv.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$o_$cv.json')); print('order', $o, 'cv', $cv, d['value'], d['phases_ms'])" >> gpurun_out/ab.txt
done; done
