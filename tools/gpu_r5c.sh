#!/bin/bash
# Round 5: LDS counters - the microbenchmark's address patterns (what SQ counts
# as a bank conflict for ds_add_u64) and the headline's scatter (pairs on),
# each counter set in its own pass
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 $GRAFT_REPO_ROOT/tools/microbench/build/lds_conflict > $GRAFT_REPO_ROOT/$OUT/r05c_lds_conflict.txt 2>&1 && echo "mb ok" &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d $GRAFT_REPO_ROOT/$OUT/r05c_mb_pmc -o mb --output-format csv -- $GRAFT_REPO_ROOT/tools/microbench/build/lds_conflict > /dev/null 2>&1 && echo "mb pmc ok" &&
cd $GRAFT_REPO_ROOT &&
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -d $PWD/$OUT/r05c_sc_pmc -o sc --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary --sync > $OUT/r05c_sc_bench.json 2> $OUT/r05c_sc_bench.err && echo "scatter pmc ok"
