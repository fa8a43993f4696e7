#!/bin/bash
# pass A with XCD-grouped rows (rows sharing H lines on one XCD) against the
# plain row-per-workgroup mapping: headline (fp64 H) and reference call (complex64 H)
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_refcall.sh default tools/variants/libcip_hip_rowsnox.so || exit 1
cat gpurun_out/ab_refcall.txt
