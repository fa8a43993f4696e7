#!/bin/bash
# Round 5: pairs opt-in build - strip / pair / c4 GPU tests, lane-kernel SQ
# counters (default, no pairs), strong C4 model at 8 ranks with the sparse all-to-all
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_strips.py tests/test_gpu_c4.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $OUT/r05f_pytest.log 2>&1 && echo "pytest ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $PWD/$OUT/r05f_sc_pmc -o sc --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary --sync > $OUT/r05f_sc_bench.json 2> $OUT/r05f_sc_bench.err && echo "pmc ok" &&
timeout -k 10 500 python tools/strong_model.py --ranks 8 > $OUT/r05f_strong_model_c4.json 2> $OUT/r05f_strong_model_c4.err && echo "model ok"
