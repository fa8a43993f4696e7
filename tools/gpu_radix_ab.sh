#!/bin/bash
# GPU suite, then CIP_RADIX_WIDE A/B (one 10-bit pass for 17-18-bit keys) at C4 (shard + strong)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/radix_pytest.log 2>&1 && echo "pytest ok" &&
BENCH_ARGS="--config c4 --no-secondary --sync" bash tools/ab_env_phases.sh CIP_RADIX_WIDE 0 1 && cp gpurun_out/ab_phases.txt gpurun_out/ab_radix_c4.txt &&
BENCH_ARGS="--config c4 --no-secondary --sync" CIP_RADIX_G1=4 bash tools/ab_env_phases.sh CIP_RADIX_WIDE 1 && cp gpurun_out/ab_phases.txt gpurun_out/ab_radix_c4_g4.txt &&
for v in 0 1; do CIP_RADIX_WIDE=$v timeout -k 10 300 python bench.py --strong --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/radix_strong_$v.json 2>> gpurun_out/radix_strong.err || exit 1; done && echo "strong ok"
