#!/bin/bash
# round 5 final tree: kernel trace of the reference call (after the FFT exchange layout) and the C4 shard line
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
R=r05as
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_${R} -o $R --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary --wstacking --single --support 6 \
    > $OUT/${R}_refcall_prof.json 2> $OUT/${R}_refcall_prof.err && echo "prof ok" &&
python3 tools/trace_summary.py $OUT/prof_${R}/${R}_kernel_trace.csv 10 $OUT/${R}_refcall_kernel_summary.md > /dev/null &&
timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline --no-secondary > $OUT/${R}_bench_c4.json 2> $OUT/${R}_bench_c4.err && echo "c4 ok"
