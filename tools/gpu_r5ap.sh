#!/bin/bash
# round 5: swizzled FFT exchange layout (CIP_FFT_XLDS=1) - FFT/imaging parity, then interleaved A/B vs the padded layout
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fft_pruned.py \
    tests/test_gpu_fft_rowskip.py tests/test_gpu_invert_parity.py tests/test_gpu_wstack_groups.py \
    tests/test_gpu_wstack_pairb.py > gpurun_out/r05ap_pytest.log 2>&1 &&
OUT=r05ap_ab_xlds REPS=3 bash tools/ab_variants.sh default ab_lib/libcip_xlds0.so &&
OUT=r05ap_ab_xlds_c4 REPS=2 BENCH_ARGS="--config c4 --no-secondary" STEPS=5 WARMUP=2 bash tools/ab_variants.sh default ab_lib/libcip_xlds0.so
