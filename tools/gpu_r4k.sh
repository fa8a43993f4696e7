export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wstack_groups.py tests/test_gpu_invert_parity.py tests/test_gpu_wplanes.py tests/test_gpu_stokes_fused.py tests/test_gpu_large_support.py tests/test_gpu_baseline_configs.py > gpurun_out/t9.log 2>&1; echo "tests rc $?" >> gpurun_out/t9.log
OUT=ab_pk REPS=2 BENCH_ARGS="--sync" bash tools/ab_variants.sh default; echo "ab rc $?"
