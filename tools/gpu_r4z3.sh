#!/bin/bash
# fp32 transforms for the packed class's complex64 planes: targeted parity
# tests first, then the reference-call A/B (fp32 at 6 waves / fp64 / fp32 with
# no occupancy target)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_grid_f32.py tests/test_gpu_baseline_configs.py tests/test_gpu_strips.py \
  > gpurun_out/r4z3_pytest.log 2>&1 || { tail -30 gpurun_out/r4z3_pytest.log; exit 1; }
tail -3 gpurun_out/r4z3_pytest.log
grep -h "max|GPU" gpurun_out/r4z3_pytest.log | head -20
REPS=2 bash tools/ab_refcall.sh default env:CIP_FFT_F32=0 tools/variants/libcip_hip_fftw1.so || exit 1
cat gpurun_out/ab_refcall.txt
