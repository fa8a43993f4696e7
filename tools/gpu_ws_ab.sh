#!/bin/bash
# w-stacking GPU tests, then the reference call A/B (current library vs tools/variants/libcip_hip_headws.so)
set -o pipefail
mkdir -p gpurun_out
L=ska-sdp-continuum-imaging-pipeline_amd/ska_sdp_cip_amd/_lib/libcip_hip.so
V=tools/variants/libcip_hip_headws.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_wstack_groups.py tests/test_gpu_invert_parity.py tests/test_gpu_baseline_configs.py tests/test_gpu_stokes_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ws_pytest.log 2>&1 && echo "pytest ok" &&
BENCH_ARGS='--wstacking --single --support 6 --no-max-err --no-secondary' STEPS=10 WARMUP=3 bash tools/ab_libs.sh $L $V $L $V && cp gpurun_out/ab_libs.txt gpurun_out/ab_ws_trim.txt
