#!/bin/bash
# Round 5: full GPU suite
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r05ak_pytest_gpu.log 2>&1 && echo ok
