#!/bin/bash
# One GPU-box pass of the round's evidence (run via gpurun from the repo root):
#   1. the -m gpu parity suite
#   2. the default bench line (C2, CPU baseline included)
#   3. rocprofv3 --kernel-trace --stats over a bench run
#   4. PMC passes (SQ issue counters + GRBM clock; FETCH_SIZE; WRITE_SIZE), each its own run
# Usage: tools/gpu_round.sh TAG [skip_tests]   -> gpurun_out/TAG/...
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${2:-}" != "skip_tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_under_rocprof.json 2> $OUT/trace.err || exit 3
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
WANT="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
HAVE=""
for c in $WANT; do grep -qw "$c" $OUT/counters_list.txt && HAVE="$HAVE $c"; done
echo "SQ counters: $HAVE"
timeout -s KILL 240 rocprofv3 --pmc $HAVE GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_sq.err || exit 4
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_fetch.err || exit 5
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_write.err || exit 6
python tools/summarize_prof.py $OUT > $OUT/summary.json || exit 7
echo done
