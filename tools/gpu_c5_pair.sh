mkdir -p gpurun_out
BENCH_ARGS='--no-max-err --no-secondary --sync' STEPS=10 WARMUP=5 bash tools/ab_libs.sh ska-sdp-continuum-imaging-pipeline_amd/ska_sdp_cip_amd/_lib/libcip_hip.so tools/variants/libcip_hip_pair5.so ska-sdp-continuum-imaging-pipeline_amd/ska_sdp_cip_amd/_lib/libcip_hip.so tools/variants/libcip_hip_pair5.so && cp gpurun_out/ab_libs.txt gpurun_out/ab_pair5.txt &&
timeout -k 10 300 python tools/bench_rows.py --mode continuum --rows 390625 --nchan 256 --npix 4096 --facets-xy 8 4 --world 8 --refcall --repeat 2 > gpurun_out/c5_refcall_w8.json 2> gpurun_out/c5.err &&
timeout -k 10 300 python tools/bench_rows.py --mode continuum --rows 390625 --nchan 256 --npix 4096 --facets-xy 8 4 --world 8 --repeat 2 > gpurun_out/c5_2d_w8.json 2>> gpurun_out/c5.err &&
timeout -k 10 400 python tools/bench_rows.py --mode continuum --rows 390625 --nchan 256 --npix 4096 --facets-xy 8 4 --world 1 --refcall --repeat 1 > gpurun_out/c5_refcall_w1.json 2>> gpurun_out/c5.err
