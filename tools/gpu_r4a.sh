export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c5.py > gpurun_out/t3.log 2>&1; echo "c5 rc $?" >> gpurun_out/t3.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r04a.json 2> gpurun_out/bench_r04a.err && \
timeout -k 10 300 python -u tools/strong_model.py --mode strips --ranks 8 > gpurun_out/strong_model_c4.json 2> gpurun_out/strong_model_c4.err && \
timeout -k 10 300 python -u tools/strong_model.py --mode wplanes --ranks 8 --single > gpurun_out/strong_model_wplanes.json 2> gpurun_out/strong_model_wplanes.err && \
timeout -k 10 200 python -u bench.py --strong --wstacking --epsilon-call --single --steps 5 --warmup 2 > gpurun_out/bench_strong_ws_n1.json 2> gpurun_out/bench_strong_ws_n1.err && \
timeout -k 10 200 python -u bench.py --support 64 --wstacking --steps 2 --warmup 1 --no-max-err --no-cpu-baseline --no-secondary --no-strong-secondary > gpurun_out/bench_c3_w64_ws.json 2> gpurun_out/bench_c3_w64_ws.err
echo "chain rc $?"
