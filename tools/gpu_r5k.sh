#!/bin/bash
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r05o -o c4o -- python3 tools/c4_phases.py > $OUT/r05o_c4_phases.json 2> $OUT/r05o.err && echo ok
