#!/bin/bash
# Round 5 close: smoke, the default bench line (CPU baseline, secondaries), the
# kernel-trace summary of the headline, the C4 shard and strong C4 lines
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROUND=r05z
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${ROUND}_smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python bench.py > $OUT/${ROUND}_bench.json 2> $OUT/${ROUND}_bench.err && echo "bench ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_${ROUND} -o $ROUND --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary > $OUT/${ROUND}_bench_prof.json 2> $OUT/${ROUND}_bench_prof.err && echo "prof ok" &&
python3 tools/trace_summary.py $OUT/prof_${ROUND}/${ROUND}_kernel_trace.csv 10 $OUT/${ROUND}_kernel_summary.md > /dev/null &&
timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline --no-secondary > $OUT/${ROUND}_bench_c4.json 2> $OUT/${ROUND}_bench_c4.err && echo "c4 ok"
