#!/bin/bash
# round 5: group pass B (CIP_WSTACK_GROUPB) - bit identity, then interleaved A/B
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wstack_pairb.py \
    > gpurun_out/r05ao_pytest.log 2>&1 &&
OUT=r05ao_ab_groupb REPS=3 bash tools/ab_variants.sh default env:CIP_WSTACK_GROUPB=1
