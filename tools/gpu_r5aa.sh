#!/bin/bash
# Round 5: faster sparse assemble; strip GPU tests; the C4 8-rank model with the assemble stage on the critical path
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_strip_exchange.py tests/test_gpu_strips.py tests/test_gpu_c4.py > $OUT/r05ae_pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 500 python tools/strong_model.py --ranks 8 > $OUT/r05ae_strong_model_c4.json 2> $OUT/r05ae_model.err && echo "model ok"
