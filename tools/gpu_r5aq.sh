#!/bin/bash
# Round 5: SQ counters of the reference call after the swizzled FFT exchange layout (one counter group)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES \
   -d $PWD/$OUT/r05aq_sq_refcall -o r05aq_sq_refcall --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-strong-secondary --sync --wstacking --single --support 6 --no-secondary --no-max-err > $OUT/r05aq_sq_refcall.json 2> $OUT/r05aq_sq_refcall.err && echo "b ok"
