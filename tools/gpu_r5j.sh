#!/bin/bash
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python tools/c4_phases.py > $OUT/r05j_c4_phases.json 2> $OUT/r05j_c4_phases.err && echo "ok"
