#!/bin/bash
# FFT column-block variants at C4 and C3 (interleaved), into gpurun_out/ab_fft_cb.txt
set -o pipefail
mkdir -p gpurun_out; rm -f gpurun_out/ab_fft_cb.txt
BASE=ska-sdp-continuum-imaging-pipeline_amd/ska_sdp_cip_amd/_lib/libcip_hip.so
for cfg in c4 c3; do
  for k in 1 2; do
    for lib in $BASE tools/variants/libcip_hip_cb16.so tools/variants/libcip_hip_cb4.so; do
      CIP_HIP_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --steps 10 --warmup 5 \
          > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
      python -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$cfg', '$lib'.split('/')[-1], d['value'], d['phases_ms'])" >> gpurun_out/ab_fft_cb.txt
    done
  done
done
