#!/bin/bash
# One parameterised GPU session (replaces the per-run gpu_r4*/gpu_r5* scripts).
# Usage: bash tools/gpu_session.sh TAG STEP [STEP ...]
# Steps (run in order, each under its own time limit, chained: the first
# failure - fault, abort, time limit - ends the session):
#   smoke            __graft_entry__.smoke()
#   pytest[=EXPR]    the -m gpu suite (EXPR: a pytest -k expression)
#   bench            the default bench line (CPU baseline, secondaries)
#   quick            bench without CPU baseline / max|err| / secondaries
#   prof             rocprofv3 kernel trace of the headline + summary
#   profrc           rocprofv3 kernel trace of the reference call (w-stacking, eps 1e-4)
#   profc4           rocprofv3 kernel trace of the C4 line (synchronous calls)
#   pmc              FETCH_SIZE / WRITE_SIZE / TCC_EA0_ATOMIC passes (synchronous steps)
#   pmcc4            FETCH_SIZE / WRITE_SIZE passes of the C4 line
#   c4               the C4 shard line
#   strong           bench --strong (C4 strong split at N = 1)
#   refcall          the reference call alone (--wstacking --single --epsilon-call)
#   ab=ENVSPEC       interleaved A/B of the quick line: ENVSPEC "K=V,K2=V2" vs the default (3 pairs)
#   abrc=ENVSPEC     the same for the reference call (w-stacking, eps 1e-4, packed class)
#   abrc2=SPEC_A;SPEC_B  two variants of the reference call against the default, interleaved
#   abc4=ENVSPEC     the same for the C4 line (one-shot calls timed synchronously too)
#   py=SCRIPT[:ARGS] python SCRIPT ARGS (tools), 300 s limit
# Output: gpurun_out/<TAG>_<step>.{log,json,md}
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
TAG=$1
shift
QUICK="--no-cpu-baseline --no-max-err --no-secondary --no-strong-secondary"
run() {  # run <limit> <name> <cmd...>: stdout to json/log, stderr to .err
  local lim=$1 name=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.out" 2> "$OUT/${TAG}_${name}.err"
  local rc=$?
  echo "step $name rc=$rc"
  return $rc
}
for step in "$@"; do
  case "$step" in
    smoke) run 300 smoke python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    pytest) run 1100 pytest python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit 1 ;;
    pytest=*) run 1100 pytest python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
                -k "${step#pytest=}" || exit 1 ;;
    bench) run 600 bench python bench.py || exit 1 ;;
    quick) run 300 quick python bench.py $QUICK || exit 1 ;;
    prof)
      run 400 prof rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof_${TAG}" -o "$TAG" --output-format csv -- \
        python3 bench.py $QUICK || exit 1
      python3 tools/trace_summary.py "$OUT/prof_${TAG}/${TAG}_kernel_trace.csv" 10 "$OUT/${TAG}_kernel_summary.md" \
        > /dev/null || exit 1 ;;
    profrc)
      run 400 profrc rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/profrc_${TAG}" -o "${TAG}rc" --output-format csv -- \
        python3 bench.py --wstacking --single --epsilon-call --sync $QUICK || exit 1
      python3 tools/trace_summary.py "$OUT/profrc_${TAG}/${TAG}rc_kernel_trace.csv" 10 \
        "$OUT/${TAG}_refcall_kernel_summary.md" > /dev/null || exit 1 ;;
    profc4)
      run 400 profc4 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/profc4_${TAG}" -o "${TAG}c4" --output-format csv -- \
        python3 bench.py --config c4 --sync --steps 6 --warmup 2 $QUICK || exit 1
      python3 tools/trace_summary.py "$OUT/profc4_${TAG}/${TAG}c4_kernel_trace.csv" 5 \
        "$OUT/${TAG}_c4_kernel_summary.md" > /dev/null || exit 1 ;;
    pmc)
      A="--steps 2 --warmup 1 --sync $QUICK"
      for c in FETCH_SIZE WRITE_SIZE TCC_EA0_ATOMIC_sum; do
        run 300 "pmc_$c" rocprofv3 --pmc $c -d "$PWD/$OUT/pmc_${TAG}_$c" -o "pmc_$c" --output-format csv -- \
          python3 bench.py $A || exit 1
      done ;;
    pmcc4)
      A="--config c4 --steps 2 --warmup 1 --sync $QUICK"
      for c in FETCH_SIZE WRITE_SIZE; do
        run 300 "pmcc4_$c" rocprofv3 --pmc $c -d "$PWD/$OUT/pmcc4_${TAG}_$c" -o "pmc_$c" --output-format csv -- \
          python3 bench.py $A || exit 1
      done ;;
    c4) run 400 c4 python bench.py --config c4 --no-cpu-baseline --no-secondary --no-strong-secondary || exit 1 ;;
    strong) run 500 strong python bench.py --strong --no-cpu-baseline || exit 1 ;;
    refcall) run 400 refcall python bench.py --wstacking --single --epsilon-call $QUICK || exit 1 ;;
    ab=*)
      spec=${step#ab=}
      sn=$(echo "$spec" | tr -c 'A-Za-z0-9\n' '_')  # the files of each ab step apart
      for i in 1 2 3; do
        run 300 "ab_${sn}_base$i" python bench.py $QUICK || exit 1
        run 300 "ab_${sn}_var$i" env ${spec//,/ } python bench.py $QUICK || exit 1
      done ;;
    abrc=*)
      spec=${step#abrc=}
      for i in 1 2 3; do
        run 300 "abrc_base$i" python bench.py --wstacking --single --epsilon-call $QUICK || exit 1
        run 300 "abrc_var$i" env ${spec//,/ } python bench.py --wstacking --single --epsilon-call $QUICK || exit 1
      done ;;
    abrc2=*)
      # two variants against the default, interleaved: abrc2=SPEC_A;SPEC_B
      spec=${step#abrc2=}
      sa=${spec%%;*}
      sb=${spec#*;}
      for i in 1 2 3; do
        run 300 "abrc2_base$i" python bench.py --wstacking --single --epsilon-call $QUICK || exit 1
        run 300 "abrc2_a$i" env ${sa//,/ } python bench.py --wstacking --single --epsilon-call $QUICK || exit 1
        run 300 "abrc2_b$i" env ${sb//,/ } python bench.py --wstacking --single --epsilon-call $QUICK || exit 1
      done ;;
    abc4=*)
      spec=${step#abc4=}
      for i in 1 2 3; do
        run 300 "abc4_base$i" python bench.py --config c4 $QUICK || exit 1
        run 300 "abc4_var$i" env ${spec//,/ } python bench.py --config c4 $QUICK || exit 1
      done ;;
    py=*)
      s=${step#py=}
      script=${s%%:*}
      args=""
      [[ "$s" == *:* ]] && args=${s#*:}
      run 300 "py_$(basename "$script" .py)" python "$script" $args || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done"
