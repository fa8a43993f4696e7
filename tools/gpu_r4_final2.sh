#!/bin/bash
# Round-4 close on the final tree: GPU suite, smoke, default bench line, headline
# kernel trace, reference-call kernel trace (each step under its own limit, && chained)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
ROUND=r04g bash tools/gpu_r4_finalA.sh &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_ref -o ref --output-format csv -- \
    python3 bench.py --sync --wstacking --single --support 6 --no-secondary --no-cpu-baseline --no-max-err \
    --no-strong-secondary --steps 5 --warmup 3 > $OUT/r04g_ref_bench.json 2> $OUT/ref_bench.err && echo "ref prof ok" &&
python3 tools/trace_summary.py $OUT/prof_ref/ref_kernel_trace.csv 5 $OUT/r04g_refcall_kernel_summary.md > /dev/null && echo "ref summary ok"
