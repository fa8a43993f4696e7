#!/bin/bash
# Round 5: kernel timeline of the pipelined headline (are plan(k+1) and scatter(k) concurrent?)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05s -o pipe -- python3 bench.py --no-cpu-baseline --no-secondary --no-max-err --steps 10 --warmup 5 > $OUT/r05s_bench.json 2> $OUT/r05s.err && echo ok
