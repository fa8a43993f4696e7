export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wstack_groups.py tests/test_gpu_invert_parity.py tests/test_gpu_wplanes.py tests/test_gpu_stokes_fused.py tests/test_gpu_flush_store.py > gpurun_out/t8.log 2>&1; echo "tests rc $?" >> gpurun_out/t8.log
STEPS=3 BENCH_ARGS="--sync --wstacking --single --support 6" bash tools/ab_env_kstats.sh CIP_GRID_F32 - 0; echo "ks rc $?"
OUT=ab_h32 REPS=2 BENCH_ARGS="--sync" bash tools/ab_variants.sh default env:CIP_GRID_F32=0; echo "ab rc $?"
