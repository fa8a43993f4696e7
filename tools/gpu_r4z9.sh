#!/bin/bash
# --single (packed class, complex64 planes, fp32 transforms) on the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --single --no-secondary --no-strong-secondary --no-cpu-baseline \
  > gpurun_out/r04g_bench_single.json 2> gpurun_out/r04g_bench_single.err && echo "single ok" &&
python -c "import json; d=json.load(open('gpurun_out/r04g_bench_single.json')); print(d['value'], d['ms_per_step'], d.get('value_sync'), d['phases_ms'], d.get('max_err'))"
