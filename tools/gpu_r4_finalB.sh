#!/bin/bash
# Round-4 close, part B: HBM traffic of the C3 scatter (one PMC counter per
# pass), SQ counters of the reference call, the C4 strong-scaling model.
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
ROUND=${ROUND:-r04}
ROUND=$ROUND bash tools/gpu_pmc.sh && python3 tools/parse_pmc.py $ROUND c3 $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_atomic > $OUT/${ROUND}_pmc_stdout.txt && cp profiles/traffic_c3.json profiles/${ROUND}_pmc_summary.md $OUT/ && echo "pmc ok" &&
TAG=sqref BENCH_ARGS="--sync --wstacking --single --support 6 --no-secondary" bash tools/gpu_sq.sh && python3 tools/sq_summary.py $OUT/sqref_a $OUT/sqref_b > $OUT/${ROUND}_sq_refcall.md && echo "sq ok" &&
timeout -k 10 400 python -u tools/strong_model.py --ranks 8 > $OUT/${ROUND}_strong_model_c4.json 2> $OUT/${ROUND}_strong_model_c4.err && echo "strong ok"
