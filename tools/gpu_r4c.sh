export TMPDIR=/tmp; mkdir -p gpurun_out
REPS=2 bash tools/ab_refcall.sh default env:CIP_WSTACK_GROUP=3 env:CIP_WSTACK_GROUP=4 tools/variants/libcip_hip_w6noflush.so; echo "ab rc $?"
TAG=sqref BENCH_ARGS="--wstacking --single --support 6 --sync --no-max-err --no-secondary" bash tools/gpu_sq.sh; echo "sq rc $?"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wstack_groups.py tests/test_gpu_wplanes.py > gpurun_out/t5.log 2>&1; echo "tests rc $?" >> gpurun_out/t5.log
