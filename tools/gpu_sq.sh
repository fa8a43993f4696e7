#!/bin/bash
# SQ counters of the kernels (diagnostic), one pass per counter group; extra
# environment settings come from the caller. TAG names the output dirs.
set -o pipefail
OUT=gpurun_out
TAG=${TAG:-sq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
   -d $PWD/$OUT/${TAG}_a -o ${TAG}_a --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong-secondary ${BENCH_ARGS:---sync} > $OUT/${TAG}_a.json 2> $OUT/${TAG}_a.err && echo "a ok" &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES \
   -d $PWD/$OUT/${TAG}_b -o ${TAG}_b --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong-secondary ${BENCH_ARGS:---sync} > $OUT/${TAG}_b.json 2> $OUT/${TAG}_b.err && echo "b ok"
