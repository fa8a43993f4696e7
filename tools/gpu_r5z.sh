#!/bin/bash
# Round 5: pipelined A/B - scatter blocks per CU beside the next call's planner (share_cus)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
OUT=r05z_ab_share_blocks REPS=2 BENCH_ARGS="--no-secondary" bash tools/ab_variants.sh default env:CIP_SHARE_BLOCKS=2 env:CIP_SCATTER_SHARE=0 && echo ok
