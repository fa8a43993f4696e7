#!/bin/bash
# Round 5: pair + strip GPU tests, bench pairs on / off, then the LDS counters
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_strips.py tests/test_gpu_invert_parity.py \
  tests/test_gpu_order_modes.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r05b_pytest.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-strong-secondary > $OUT/r05b_bench.json 2> $OUT/r05b_bench.err &&
echo "bench ok" &&
CIP_PAIRS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-strong-secondary --no-max-err > $OUT/r05b_bench_nopairs.json 2> $OUT/r05b_bench_nopairs.err &&
echo "bench nopairs ok" &&
bash tools/gpu_r5c.sh
