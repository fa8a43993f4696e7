export TMPDIR=/tmp; mkdir -p gpurun_out
OUT=ab_f32b REPS=2 BENCH_ARGS="--sync" bash tools/ab_variants.sh default env:CIP_GRID_F32=0; echo "ab rc $?"
OUT=ab_f32b_single REPS=2 BENCH_ARGS="--single --no-secondary" bash tools/ab_variants.sh default env:CIP_GRID_F32=0; echo "ab2 rc $?"
timeout -k 10 400 python -u tools/strong_model.py --ranks 8 > gpurun_out/strong_c4_cost.json 2> gpurun_out/strong_c4_cost.err; echo "strong rc $?"
