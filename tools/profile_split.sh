#!/bin/bash
export TMPDIR=/tmp
OUT=gpurun_out/prof2
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I rust-bitcoinconsensus_amd/csrc tools/fe_bench.hip -o tools/_build/fe_bench.so || exit 5
timeout -k 10 120 python tools/fe_bench_run.py > $OUT/fe_bench.txt 2>&1 || exit 6
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit 1
echo done
