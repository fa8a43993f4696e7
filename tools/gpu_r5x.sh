#!/bin/bash
# Round 5: place pass templated on the row mode (dense: 71 VGPRs, 7 waves) vs the previous build, and at 8 waves
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
OUT=r05x_ab_place_rm REPS=2 bash tools/ab_variants.sh default tools/variants/libcip_hip_prevplace.so tools/variants/libcip_hip_placew8.so && echo ok
