export TMPDIR=/tmp; mkdir -p gpurun_out
OUT=ab_radix REPS=3 BENCH_ARGS="--sync --no-secondary" bash tools/ab_variants.sh default tools/variants/libcip_hip_rw5.so tools/variants/libcip_hip_rw6.so; echo "ab rc $?"
STEPS=5 BENCH_ARGS="--sync --no-secondary --no-strong-secondary" CIP_HIP_LIB=$PWD/tools/variants/libcip_hip_rw6.so bash tools/ab_env_kstats.sh CIP_DUMMY rw6; echo "ks rc $?"
