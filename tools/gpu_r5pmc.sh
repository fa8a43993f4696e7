#!/bin/bash
# Round 5: HBM traffic of the C3 headline kernels, one PMC counter per pass
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950); synchronous
# calls, no secondaries, no max|err| sample (one scatter variant in the trace)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --sync --no-secondary --no-strong-secondary --no-max-err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $PWD/$OUT/pmc_r05_fetch -o r05_fetch --output-format csv -- \
    python3 bench.py $ARGS > $OUT/pmc_r05_fetch.json 2> $OUT/pmc_r05_fetch.err && echo "fetch ok" &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $PWD/$OUT/pmc_r05_write -o r05_write --output-format csv -- \
    python3 bench.py $ARGS > $OUT/pmc_r05_write.json 2> $OUT/pmc_r05_write.err && echo "write ok" &&
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d $PWD/$OUT/pmc_r05_atomic -o r05_atomic --output-format csv -- \
    python3 bench.py $ARGS > $OUT/pmc_r05_atomic.json 2> $OUT/pmc_r05_atomic.err && echo "atomic ok"
