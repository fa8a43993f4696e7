export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_strips.py > gpurun_out/t13.log 2>&1; echo "tests rc $?" >> gpurun_out/t13.log
timeout -k 10 600 python -u tools/strong_model.py --mode wstrips --single --ranks 8 --steps 2 > gpurun_out/wstrips_single2.json 2> gpurun_out/wstrips_single2.err; echo "wstrips rc $?"
timeout -k 10 600 python -u tools/strong_model.py --mode wplanes --single --ranks 8 --steps 2 > gpurun_out/wplanes_single2.json 2> gpurun_out/wplanes_single2.err; echo "wplanes rc $?"
