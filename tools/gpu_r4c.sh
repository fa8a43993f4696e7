export TMPDIR=/tmp; mkdir -p gpurun_out
REPS=2 bash tools/ab_refcall.sh default tools/variants/libcip_hip_w6noflush.so; echo "ab rc $?"
TAG=sqref BENCH_ARGS="--wstacking --single --support 6 --sync --no-max-err --no-secondary" bash tools/gpu_sq.sh; echo "sq rc $?"
