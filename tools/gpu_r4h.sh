export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=sqref BENCH_ARGS="--sync --wstacking --single --support 6 --no-secondary" bash tools/gpu_sq.sh && python3 tools/sq_summary.py gpurun_out/sqref_a gpurun_out/sqref_b > gpurun_out/sqref_summary.md; echo "sq rc $?"
