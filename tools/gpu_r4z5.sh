#!/bin/bash
# w screen of fp32 transforms: fp32 sine / cosine after an exact fp64 phase
# reduction (default) vs fp64 sincospi vs no screen (ablation); then the
# single-class parity tests on the default build
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_refcall.sh default tools/variants/libcip_hip_scr64.so tools/variants/libcip_hip_scrabl.so || exit 1
cat gpurun_out/ab_refcall.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_grid_f32.py tests/test_gpu_baseline_configs.py tests/test_gpu_strips.py \
  > gpurun_out/r4z5_pytest.log 2>&1 || { tail -30 gpurun_out/r4z5_pytest.log; exit 1; }
tail -3 gpurun_out/r4z5_pytest.log
grep -h "single" gpurun_out/r4z5_pytest.log | grep -i "err" | head
