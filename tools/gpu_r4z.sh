#!/bin/bash
# fused multi-plane flush: A/B on the reference call (old per-plane flush as a
# variant library), then the GPU suite on the new in-tree build
set -o pipefail
mkdir -p gpurun_out
REPS=2 bash tools/ab_refcall.sh default tools/variants/libcip_hip_oldflush.so || exit 1
cat gpurun_out/ab_refcall.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4z_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r4z_pytest.log
exit $rc
