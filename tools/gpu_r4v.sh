export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config c4 --no-cpu-baseline --no-secondary --no-strong-secondary > gpurun_out/r04_c4.json 2> gpurun_out/r04_c4.err; echo "c4 rc $?"
timeout -k 10 400 python -u bench.py --single --no-cpu-baseline --no-secondary --no-strong-secondary > gpurun_out/r04_single.json 2> gpurun_out/r04_single.err; echo "single rc $?"
