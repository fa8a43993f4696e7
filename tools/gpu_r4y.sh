export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_strips.py -k masked > gpurun_out/t14.log 2>&1; echo "tests rc $?" >> gpurun_out/t14.log
