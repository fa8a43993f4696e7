#!/bin/bash
# Kernel-trace stats per environment setting: tools/ab_env_kstats.sh VAR val1 val2 ... ("-" = unset)
# BENCH_ARGS: bench.py arguments (default --sync) -> gpurun_out/ks_<VAR>_<val>/ and gpurun_out/kstats.txt
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/kstats.txt
var=$1; shift
for v in "$@"; do
  if [ "$v" = "-" ]; then unset $var; else export $var=$v; fi
  name=${var}_${v}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/ks_$name -o ks --output-format csv \
    -- python3 bench.py --steps ${STEPS:-5} --warmup 3 --no-cpu-baseline --no-max-err --no-secondary ${BENCH_ARGS:---sync} \
    > gpurun_out/ks_$name.json 2> gpurun_out/ks_$name.err || exit 1
  python3 tools/kstats.py $name gpurun_out/ks_$name >> gpurun_out/kstats.txt || exit 1
done
