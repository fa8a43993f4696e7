#!/bin/bash
# Round 5, first GPU session: the changed / new GPU tests (masked strip pass A
# at W = 48 / 64, the full C4 8-strip emulation vs one-shot), then the strong
# C4 bench at N = 1 with its new DFT-pixel parity, then the default bench line
# (reduced-image parity) without the CPU baseline.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_strips.py tests/test_gpu_c4.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $OUT/r05a_pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --strong --steps 5 --warmup 2 > $OUT/r05a_strong.json 2> $OUT/r05a_strong.err &&
echo "strong ok" &&
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/r05a_bench.json 2> $OUT/r05a_bench.err && echo "bench ok"
