#!/bin/bash
# HBM traffic of the kernels from PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ROUND=${ROUND:-r01}
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $PWD/$OUT/pmc_fetch -o ${ROUND}_fetch --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:---sync} > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err && echo "fetch ok" &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $PWD/$OUT/pmc_write -o ${ROUND}_write --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:---sync} > $OUT/pmc_write.json 2> $OUT/pmc_write.err && echo "write ok" &&
timeout -k 10 600 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d $PWD/$OUT/pmc_atomic -o ${ROUND}_atomic --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:---sync} > $OUT/pmc_atomic.json 2> $OUT/pmc_atomic.err && echo "atomic ok"
