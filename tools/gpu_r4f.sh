export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS=3 BENCH_ARGS="--sync --wstacking --single --support 6" bash tools/ab_env_kstats.sh CIP_GRID_F32 - 0; echo "ks rc $?"
