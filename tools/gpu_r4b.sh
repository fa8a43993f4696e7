export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_invert_parity.py tests/test_gpu_stokes_fused.py tests/test_gpu_wstack_groups.py tests/test_gpu_wplanes.py tests/test_gpu_flush_store.py tests/test_gpu_baseline_configs.py::test_c2_full_reference_call_wstacking tests/test_gpu_c5.py > gpurun_out/t4.log 2>&1; echo "tests rc $?" >> gpurun_out/t4.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-strong-secondary > gpurun_out/bench_r04b.json 2> gpurun_out/bench_r04b.err
timeout -k 10 300 python -u bench.py --single --no-cpu-baseline --no-strong-secondary > gpurun_out/bench_r04b_single.json 2> gpurun_out/bench_r04b_single.err
echo done
