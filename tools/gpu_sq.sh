#!/bin/bash
# SQ counters of the scatter kernel (diagnostic), one pass per counter group.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
   -d $PWD/$OUT/sq_a -o sq_a --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq_a.json 2> $OUT/sq_a.err && echo "a ok" &&
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES \
   -d $PWD/$OUT/sq_b -o sq_b --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq_b.json 2> $OUT/sq_b.err && echo "b ok"
