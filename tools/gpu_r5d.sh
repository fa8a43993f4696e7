#!/bin/bash
# Round 5: pairs after the register fixes - tests, bench on/off, kernel trace, SQ counters
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_invert_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $OUT/r05d_pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-strong-secondary > $OUT/r05d_bench.json 2> $OUT/r05d_bench.err &&
echo "bench ok" &&
CIP_PAIRS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-strong-secondary --no-max-err > $OUT/r05d_bench_nopairs.json 2> $OUT/r05d_bench_nopairs.err &&
echo "bench nopairs ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/r05d_prof -o r05d --output-format csv -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary --sync > $OUT/r05d_prof_bench.json 2> $OUT/r05d_prof_bench.err && echo "trace ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $PWD/$OUT/r05d_sc_pmc -o sc --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary --sync > $OUT/r05d_sc_bench.json 2> $OUT/r05d_sc_bench.err && echo "pmc ok"
