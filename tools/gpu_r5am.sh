#!/bin/bash
# Round 5: float plane accumulator - its tests, then interleaved A/B on the reference call
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_wstack_pairb.py > $OUT/r05am_pytest.log 2>&1 && echo "pytest ok" &&
OUT=r05am_ab_wacc REPS=2 bash tools/ab_variants.sh default env:CIP_WACC_F32=0 && echo ok
