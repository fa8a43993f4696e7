#!/bin/bash
# Round 5: interleaved pipeline A/B - place pass at 8 waves/SIMD (64 VGPRs) beside the scatter
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_api_validation.py > $OUT/r05u_pytest.log 2>&1 && \
OUT=r05u_ab_placew8 REPS=3 BENCH_ARGS="--no-secondary" bash tools/ab_variants.sh default tools/variants/libcip_hip_placew8.so && echo ok
