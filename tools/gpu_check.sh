#!/bin/bash
# Iteration loop on the GPU box (run via gpurun): parity tests, bench (no CPU leg), kernel trace.
#   gpurun --timeout 900 -- bash tools/gpu_check.sh TAG
export TMPDIR=/tmp
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit 3
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \;
