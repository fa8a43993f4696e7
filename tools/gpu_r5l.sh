#!/bin/bash
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_strips.py tests/test_gpu_order_modes.py tests/test_gpu_flush_store.py tests/test_gpu_large_support.py tests/test_gpu_streaming.py tests/test_gpu_tiling_and_api.py tests/test_gpu_invert_parity.py tests/test_gpu_c4.py > $OUT/r05n_pytest.log 2>&1 && \
timeout -k 10 300 python tools/c4_phases.py > $OUT/r05n_c4_phases.json 2> $OUT/r05n_c4_phases.err && CIP_PACKED_RUNS=0 timeout -k 10 300 python tools/c4_phases.py > $OUT/r05n_c4_phases_nopk.json 2>> $OUT/r05n_c4_phases.err && echo ok
