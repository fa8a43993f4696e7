#!/bin/bash
# kernel trace of the reference call alone (C3, W = 6, w-stacking, single)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_ref -o ref --output-format csv -- \
    python3 bench.py --sync --wstacking --single --support 6 --no-secondary --no-cpu-baseline --no-max-err \
    --no-strong-secondary --steps 5 --warmup 3 > $OUT/ref_bench.json 2> $OUT/ref_bench.err && echo "prof ok" &&
python3 tools/trace_summary.py $OUT/prof_ref/ref_kernel_trace.csv 5 $OUT/r04_refcall_kernel_summary.md > /dev/null && echo "summary ok"
