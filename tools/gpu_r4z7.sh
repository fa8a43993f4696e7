#!/bin/bash
# pass B accumulator preload (default) vs load-after-transform; then the
# w-stacking parity tests and the reference call's kernel trace
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
REPS=2 bash tools/ab_refcall.sh default tools/variants/libcip_hip_nopre.so || exit 1
cat $OUT/ab_refcall.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_grid_f32.py tests/test_gpu_baseline_configs.py tests/test_gpu_strips.py tests/test_gpu_wstack_groups.py tests/test_gpu_wplanes.py tests/test_gpu_invert_parity.py tests/test_gpu_fft_pruned.py \
  > $OUT/r4z7_pytest.log 2>&1 || { tail -30 $OUT/r4z7_pytest.log; exit 1; }
tail -2 $OUT/r4z7_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_ref -o ref --output-format csv -- \
    python3 bench.py --sync --wstacking --single --support 6 --no-secondary --no-cpu-baseline --no-max-err \
    --no-strong-secondary --steps 5 --warmup 3 > $OUT/ref_bench.json 2> $OUT/ref_bench.err && echo "prof ok" &&
python3 tools/trace_summary.py $OUT/prof_ref/ref_kernel_trace.csv 5 $OUT/r04_refcall_kernel_summary.md > /dev/null && echo "summary ok"
