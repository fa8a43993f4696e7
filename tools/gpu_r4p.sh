export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_grid_f32.py > gpurun_out/t11.log 2>&1; echo "tests rc $?" >> gpurun_out/t11.log
OUT=ab_ow REPS=3 BENCH_ARGS="--no-secondary" bash tools/ab_variants.sh default tools/variants/libcip_hip_ow2048.so; echo "ab rc $?"
