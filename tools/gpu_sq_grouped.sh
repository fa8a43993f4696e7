set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
TAG=sqg BENCH_ARGS="--sync --no-max-err" bash tools/gpu_sq.sh &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-max-err --support 6 > $OUT/bench_g6.json 2> $OUT/bench_g6.err && echo "g6 ok" &&
CIP_GROUPED=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-max-err --support 6 > $OUT/bench_l6.json 2> $OUT/bench_l6.err && echo "l6 ok"
