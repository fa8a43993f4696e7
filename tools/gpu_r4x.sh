export TMPDIR=/tmp; mkdir -p gpurun_out
CIP_HIP_LIB=$PWD/tools/variants/libcip_hip_kb.so timeout -k 10 300 python -u tools/kblocks.py > gpurun_out/kblocks.json 2> gpurun_out/kblocks.err; echo "kb rc $?"
