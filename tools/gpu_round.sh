#!/bin/bash
# One GPU session: parity tests (incl. the BASELINE-config whole-image tests),
# smoke, bench (with max|err| and the CPU baseline), kernel-trace profile.
# Every GPU step has its own time limit; steps are chained with && so the
# first failure (fault, abort, timeout) ends the session.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROUND=${ROUND:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && echo "bench ok" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o $ROUND --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-max-err --no-secondary > $OUT/bench_prof.json 2> $OUT/bench_prof.err && echo "prof ok" &&
python3 tools/trace_summary.py $OUT/prof/${ROUND}_kernel_trace.csv 10 $OUT/${ROUND}_kernel_summary.md > /dev/null &&
timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err && echo "c4 ok" &&
timeout -k 10 400 python bench.py --strong --no-cpu-baseline > $OUT/bench_strong.json 2> $OUT/bench_strong.err && echo "strong ok"
