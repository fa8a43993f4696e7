#!/bin/bash
# Round 5: float plane accumulator of the packed class - full GPU suite, then interleaved A/B
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05al_pytest_gpu.log 2>&1 && echo "pytest ok" &&
OUT=r05al_ab_wacc REPS=2 bash tools/ab_variants.sh default env:CIP_WACC_F32=0 && echo ok
