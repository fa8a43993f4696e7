#!/bin/bash
# plane-group unit of 768 threads (12 waves; 2 units per CU = 24 waves) against 512
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_refcall.sh default tools/variants/libcip_hip_gt768.so || exit 1
cat gpurun_out/ab_refcall.txt
