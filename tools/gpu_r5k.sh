#!/bin/bash
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/r05m -o c4m -- python3 tools/c4_phases.py > $OUT/r05m_c4_phases.json 2> $OUT/r05m.err && echo ok
