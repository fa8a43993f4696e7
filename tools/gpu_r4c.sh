export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_invert_parity.py tests/test_gpu_tiling_and_api.py tests/test_gpu_strips.py tests/test_gpu_wstack_groups.py tests/test_gpu_order_modes.py > gpurun_out/t5.log 2>&1; echo "tests rc $?" >> gpurun_out/t5.log
OUT=ab_order REPS=2 bash tools/ab_variants.sh default env:CIP_ORDER_CLASS=gather env:CIP_PLACE_SPLIT=1 tools/variants/libcip_hip_placeabl4.so; echo "ab1 rc $?"
OUT=ab_refg REPS=2 BENCH_ARGS="--sync" bash tools/ab_variants.sh default env:CIP_WSTACK_GROUP=3 env:CIP_WSTACK_GROUP=4 tools/variants/libcip_hip_w6noflush.so; echo "ab2 rc $?"
TAG=sqref BENCH_ARGS="--wstacking --single --support 6 --sync --no-max-err --no-secondary" bash tools/gpu_sq.sh; echo "sq rc $?"
