#!/bin/bash
# GPU tests (full report) + a short bench per CIP_* env setting given as args.
# Stops at the first abort / fault / timeout of a GPU step.
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab.txt
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/ab.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures; anything else = crash
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_one.json 2>gpurun_out/ab_err.log || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$cfg', d['value'], d['phases_ms'])" >> gpurun_out/ab.txt
done
[ $rc -eq 0 ]
