#!/bin/bash
# Round-4 close, part A: the whole -m gpu suite, smoke, the default bench line
# and its kernel-trace profile (each GPU step under its own limit, && chained).
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
ROUND=${ROUND:-r04}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/${ROUND}_pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${ROUND}_smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python bench.py > $OUT/${ROUND}_bench.json 2> $OUT/${ROUND}_bench.err && echo "bench ok" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_${ROUND} -o ${ROUND} --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary > $OUT/${ROUND}_bench_prof.json 2> $OUT/${ROUND}_bench_prof.err && echo "prof ok" &&
python3 tools/trace_summary.py $OUT/prof_${ROUND}/${ROUND}_kernel_trace.csv 10 $OUT/${ROUND}_kernel_summary.md > /dev/null && echo "summary ok"
