#!/bin/bash
# fp32 pass A compiled for 6 / 8 waves per SIMD (three / four workgroups per CU) vs unconstrained
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_refcall.sh default tools/variants/libcip_hip_rows6.so tools/variants/libcip_hip_rows8.so || exit 1
cat gpurun_out/ab_refcall.txt
