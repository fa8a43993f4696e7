#!/bin/bash
# round 5: packed-class plane groups of 14 (CIP_WSTACK_GROUP=14, one block per CU) - parity, then interleaved A/B of the reference call
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wstack_groups.py \
    > gpurun_out/r05at_pytest.log 2>&1 &&
OUT=r05at_ab_g14 REPS=3 bash tools/ab_variants.sh default env:CIP_WSTACK_GROUP=14
