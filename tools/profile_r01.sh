#!/bin/bash
# rocprofv3 kernel-trace + PMC passes over bench.py (run on the GPU box via gpurun)
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --n 262144 --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_fetch.err || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --n 262144 --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_write.err || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python bench.py --n 262144 --steps 1 --warmup 0 --no-cpu > /dev/null 2> $OUT/pmc_sq.err || exit 4
echo done
