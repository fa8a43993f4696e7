#!/bin/bash
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_strips.py tests/test_gpu_tiling_and_api.py > $OUT/r05p_pytest.log 2>&1 && \
timeout -k 10 300 python tools/c4_phases.py > $OUT/r05p_c4_phases.json 2> $OUT/r05p_c4_phases.err && echo ok
