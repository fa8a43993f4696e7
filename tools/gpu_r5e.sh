#!/bin/bash
# Round 5: tap-bias variant (CIP_TAP_BIAS=1 scatter build) parity + interleaved A/B
# against the default build, pairs on / off
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
V=$PWD/tools/variants/libcip_hip_bias.so
CIP_HIP_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_invert_parity.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $OUT/r05e_pytest_bias.log 2>&1 && echo "pytest bias ok" || exit 1
rm -f $OUT/r05e_ab.txt
for rep in 1 2; do
  for lib in default $V; do
    for pairs in 0 1; do
      if [ "$lib" = default ]; then unset CIP_HIP_LIB; else export CIP_HIP_LIB=$lib; fi
      CIP_PAIRS=$pairs timeout -k 10 200 python bench.py --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary \
        > $OUT/r05e_one.json 2> $OUT/r05e_err.log || exit 1
      python -c "import json; d=json.load(open('$OUT/r05e_one.json')); print('$(basename $lib) pairs=$pairs', d['value'], d['ms_per_step'], d['value_sync'], d['phases_ms'])" >> $OUT/r05e_ab.txt
    done
  done
done
unset CIP_HIP_LIB
echo "ab ok"
