#!/bin/bash
# GPU suite (incl. the forced-store parity test), C4 shard bench with max|err| (stores on at 16384^2), strong C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/store_pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 400 python bench.py --config c4 --no-cpu-baseline > gpurun_out/store_c4.json 2> gpurun_out/store_c4.err && echo "c4 ok" &&
timeout -k 10 400 python bench.py --strong --no-cpu-baseline > gpurun_out/store_strong.json 2> gpurun_out/store_strong.err && echo "strong ok"
