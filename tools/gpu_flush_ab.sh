#!/bin/bash
# GPU suite, then CIP_FLUSH_STORE A/B (sole-unit private-cell stores) at C4 and C3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/flush_pytest.log 2>&1 && echo "pytest ok" &&
BENCH_ARGS="--config c4 --no-secondary --sync" bash tools/ab_env_phases.sh CIP_FLUSH_STORE 0 1 && cp gpurun_out/ab_phases.txt gpurun_out/ab_flush_c4.txt &&
BENCH_ARGS="--no-secondary" bash tools/ab_env_phases.sh CIP_FLUSH_STORE 0 1 && cp gpurun_out/ab_phases.txt gpurun_out/ab_flush_c3.txt
