export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS=5 BENCH_ARGS="--sync --no-strong-secondary" bash tools/ab_env_kstats.sh CIP_DUMMY - ; echo "ks rc $?"
