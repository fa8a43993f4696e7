#!/bin/bash
# A/B kernel-trace profiles: the default build/env ("a") and one env setting ("b").
# usage: bash tools/gpu_ab.sh VAR=value [bench args...]
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
AB="$1"; shift
rm -rf $OUT/prof_a $OUT/prof_b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_a -o prof --output-format csv -- \
    python3 bench.py --steps 10 --warmup 10 --no-cpu-baseline "$@" > $OUT/ab_a.json 2> $OUT/ab_a.err && echo "a ok" &&
export "$AB" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_b -o prof --output-format csv -- \
    python3 bench.py --steps 10 --warmup 10 --no-cpu-baseline "$@" > $OUT/ab_b.json 2> $OUT/ab_b.err && echo "b ok"
