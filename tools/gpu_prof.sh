#!/bin/bash
# Kernel-trace profile of a short bench run only (per-kernel durations).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
rm -rf $OUT/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o prof --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench_prof.json 2> $OUT/bench_prof.err && echo "prof ok"
