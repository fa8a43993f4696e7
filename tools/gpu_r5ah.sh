#!/bin/bash
# Round 5: plane groups of 6 / 7 packed sub-grids (two blocks per CU) for the reference call - parity, then A/B
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
CIP_WSTACK_GROUP=7 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wstack_groups.py tests/test_gpu_invert_parity.py > $OUT/r05ah_pytest_g7.log 2>&1 && echo "g7 parity ok" &&
OUT=r05ah_ab_wstack_group REPS=2 bash tools/ab_variants.sh default env:CIP_WSTACK_GROUP=6 env:CIP_WSTACK_GROUP=7 && echo ok
