#!/bin/bash
# Round 5: interleaved pipeline A/B - plan-stream priority (and the plan-stream scatter under it)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
OUT=r05v_ab_plan_priority REPS=2 BENCH_ARGS="--no-secondary" bash tools/ab_variants.sh default env:CIP_PLAN_PRIORITY=high env:CIP_PLAN_PRIORITY=low && echo ok
