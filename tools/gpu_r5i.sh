#!/bin/bash
# Round 5: plane-pair pass B (CIP_WSTACK_PAIRB) parity + refcall A/B
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wstack_pairb.py -m gpu -x -v -s --timeout 240 --timeout-method thread \
  > $OUT/r05i_pytest.log 2>&1 && echo "pytest ok" || exit 1
rm -f $OUT/r05i_ab.txt
for rep in 1 2; do
  for pb in 0 1; do
    CIP_WSTACK_PAIRB=$pb timeout -k 10 200 python bench.py --no-cpu-baseline --no-max-err --no-strong-secondary --steps 10 \
      > $OUT/r05i_one.json 2> $OUT/r05i_err.log || exit 1
    python -c "import json; d=json.load(open('$OUT/r05i_one.json')); r=d['secondary']['reference_call']; print('pairb=$pb', r['value'], r['ms_per_step'], r['phases_ms_sync'])" >> $OUT/r05i_ab.txt
  done
done
echo "ab ok"
