#!/bin/bash
# Interleaved A/B of bench.py variants (${REPS:-2} rounds): each arg is
# "default" (the in-tree build), a library path (CIP_HIP_LIB) or
# "env:NAME=VALUE" (an environment switch on the in-tree build). One line per
# run into gpurun_out/${OUT:-ab_variants}.txt: variant, headline value, phases
# (and the reference call's value / phases when the run reports it).
# BENCH_ARGS is appended to the bench command.
mkdir -p gpurun_out; OUTF=gpurun_out/${OUT:-ab_variants}.txt; rm -f $OUTF
for rep in $(seq ${REPS:-2}); do
  for v in "$@"; do
    (
      case "$v" in
        default) ;;
        env:*) export "${v#env:}" ;;
        *) export CIP_HIP_LIB=$v ;;
      esac
      timeout -k 10 240 python bench.py --no-cpu-baseline --no-strong-secondary --no-max-err --steps ${STEPS:-10} \
          --warmup ${WARMUP:-5} ${BENCH_ARGS} > gpurun_out/ab_one.json 2> gpurun_out/ab_err.log || exit 1
      python -c "
import json; d=json.load(open('gpurun_out/ab_one.json')); r=d.get('secondary', {}).get('reference_call')
print('$v', d['value'], d['phases_ms'], '' if r is None else ('refcall %s %s' % (r['value'], r['phases_ms_sync'])))" >> $OUTF
    ) || exit 1
  done
done
