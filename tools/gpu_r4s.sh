export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --strong --wstacking --epsilon-call --single --steps 3 --warmup 1 > gpurun_out/bench_wstrips_n1.json 2> gpurun_out/bench_wstrips_n1.err; echo "bench wstrips rc $?"
