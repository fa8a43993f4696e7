#!/bin/bash
# Grouped-scatter check: parity tests, then the bench with and without it.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/microbench/build/valu_ops > $OUT/valu_ops.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_invert_parity.py tests/test_gpu_baseline_configs.py tests/test_gpu_full_size.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_grouped.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_grouped.json 2> $OUT/bench_grouped.err && echo "bench grouped ok" &&
CIP_GROUPED=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-max-err > $OUT/bench_lane.json 2> $OUT/bench_lane.err && echo "bench lane ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/profg -o grp --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-max-err > $OUT/bench_gprof.json 2> $OUT/bench_gprof.err && echo "prof ok" &&
python3 tools/trace_summary.py $OUT/profg/grp_kernel_trace.csv 10 $OUT/grp_kernel_summary.md > /dev/null
[ -n "$SQ" ] && TAG=sqg BENCH_ARGS="--sync --no-max-err" bash tools/gpu_sq.sh
true
