export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wstack_groups.py tests/test_gpu_invert_parity.py tests/test_gpu_wplanes.py tests/test_gpu_stokes_fused.py tests/test_gpu_flush_store.py tests/test_gpu_order_modes.py > gpurun_out/t10.log 2>&1; echo "tests rc $?" >> gpurun_out/t10.log
OUT=ab_fold REPS=2 BENCH_ARGS="--sync" bash tools/ab_variants.sh default tools/variants/libcip_hip_nofold.so env:CIP_PACKED_PIECES=1; echo "ab rc $?"
OUT=ab_fold_single REPS=2 BENCH_ARGS="--single --no-secondary" bash tools/ab_variants.sh default tools/variants/libcip_hip_nofold.so; echo "ab2 rc $?"
