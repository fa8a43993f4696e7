#!/bin/bash
# Round 5 close: full GPU suite, smoke and the default bench line on the final tree
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05au_pytest_gpu.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r05au_smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python bench.py > $OUT/r05au_bench.json 2> $OUT/r05au_bench.err && echo "bench ok"
