#!/bin/bash
# One parameterised GPU call (run via gpurun) instead of one-off launchers: each STEP runs under its
# own time limit, output under gpurun_out/TAG/, and the first failing step ends the call.
#   tools/gpu_run.sh TAG STEP...
#   STEP: tests[=PYTEST_K_EXPR]   pytest -m gpu (optionally -k EXPR)        -> pytest_gpu.log
#         smoke                   __graft_entry__.smoke()                  -> smoke.log
#         bench[=ARGS]            python bench.py ARGS (',' for spaces)    -> bench_N.json / .err
#         dropin[=N,CALLS]        tools/dropin_e2e.py (drop-in alone)      -> dropin.txt
#         prof=CONFIG             tools/profile_c2.sh-style trace of one bench config
set -o pipefail
export TMPDIR=/tmp
T=${1:?tag}; shift
O=gpurun_out/$T
mkdir -p $O
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
      tail -2 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
        || { tail -20 $O/smoke.log; exit 2; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${arg//,/ } > $O/bench_$i.json 2> $O/bench_$i.err \
        || { tail -20 $O/bench_$i.err; exit 3; }
      python3 tools/bench_summary.py $O/bench_$i.json ;;
    dropin)
      a=${arg//,/ }
      timeout -k 10 300 python3 tools/dropin_e2e.py ${a:-1000000 20} >> $O/dropin.txt 2>&1 \
        || { tail -20 $O/dropin.txt; exit 4; }
      tail -1 $O/dropin.txt ;;
    prof)
      mkdir -p $O/prof_$arg
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$arg -o run -- \
        python3 bench.py --config $arg --no-extra --no-cpu --steps 10 --warmup 3 --sustain-s 0 \
        > $O/prof_$arg/bench.json 2> $O/prof_$arg/bench.err || { tail -20 $O/prof_$arg/bench.err; exit 5; } ;;
    *) echo "unknown step $step"; exit 9 ;;
  esac
done
