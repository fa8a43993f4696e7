#!/bin/bash
# Box probe: hardware + what is importable (ducc0 decides the CPU baseline kind).
set -o pipefail
mkdir -p gpurun_out
{
  echo "== nproc: $(nproc)  affinity: $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"
  lscpu | grep -E "Model name|Socket|Thread|Core" ;
  python3 -c "import ducc0; print('ducc0', ducc0.__version__)" 2>&1 | tail -1
  rocminfo | grep -E "Marketing Name|Compute Unit|gfx950" | head -6
  free -g | head -2
} > gpurun_out/probe.txt 2>&1
timeout -k 10 120 ./tools/microbench/build/lds_atomics > gpurun_out/lds_atomics.txt 2>&1
