#!/bin/bash
# Round 5: plan-stream scatter for pipelined 2-D calls - parity, then interleaved A/B
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_api_validation.py tests/test_gpu_stokes_fused.py "tests/test_gpu_full_size.py::test_c3_pipelined_calls_equal_synchronous" > $OUT/r05t_pytest.log 2>&1 && \
OUT=r05t_ab_pipe_scatter REPS=3 BENCH_ARGS="--no-secondary" bash tools/ab_variants.sh default env:CIP_PIPE_SCATTER=0 && echo ok
