#!/bin/bash
# HBM traffic of the C3 headline's kernels alone (no secondary measurements in the run)
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
ROUND=${ROUND:-r04}
rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_atomic
ROUND=$ROUND BENCH_ARGS="--sync --no-secondary --no-strong-secondary" bash tools/gpu_pmc.sh && python3 tools/parse_pmc.py $ROUND c3 $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_atomic > $OUT/${ROUND}_pmc_stdout.txt && cp profiles/traffic_c3.json profiles/${ROUND}_pmc_summary.md $OUT/ && echo "pmc ok"
