export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_strips.py tests/test_gpu_workspace_state.py > gpurun_out/t12.log 2>&1; echo "tests rc $?" >> gpurun_out/t12.log
timeout -k 10 600 python -u tools/strong_model.py --mode wstrips --single --ranks 8 --steps 2 > gpurun_out/wstrips_single.json 2> gpurun_out/wstrips_single.err; echo "wstrips rc $?"
timeout -k 10 500 python -u tools/strong_model.py --ranks 8 --steps 2 > gpurun_out/strips_masked.json 2> gpurun_out/strips_masked.err; echo "strips rc $?"
