export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_invert_parity.py tests/test_gpu_wstack_groups.py tests/test_gpu_order_modes.py tests/test_gpu_stokes_fused.py tests/test_gpu_baseline_configs.py::test_c2_full_reference_call_wstacking tests/test_gpu_workspace_state.py > gpurun_out/t6.log 2>&1; echo "tests rc $?" >> gpurun_out/t6.log
OUT=ab_f32 REPS=2 BENCH_ARGS="--sync" bash tools/ab_variants.sh default env:CIP_GRID_F32=0 env:CIP_FLUSH_STORE=1 tools/variants/libcip_hip_w6noflush.so; echo "ab rc $?"
OUT=ab_f32_single REPS=2 BENCH_ARGS="--single --no-secondary" bash tools/ab_variants.sh default env:CIP_GRID_F32=0; echo "ab2 rc $?"
