#!/bin/bash
# rocprofv3 evidence for one bench config (run on the GPU box via gpurun):
#   trace: --kernel-trace --stats over the bench command itself (bench line printed alongside)
#   fetch / write: separate --pmc FETCH_SIZE and WRITE_SIZE passes (one TCC group each) over a
#   one-step run of the same workload
# Usage: tools/profile_round.sh TAG CONFIG [N]   -> gpurun_out/TAG/...
export TMPDIR=/tmp
TAG=${1:-prof}
CFG=${2:-c2}
N=${3:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
NA=""
[ -n "$N" ] && NA="--n $N"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --config $CFG $NA --steps 5 --warmup 2 --no-cpu --sustain-s 0 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --config $CFG $NA --steps 1 --warmup 0 --no-cpu --sustain-s 0 > /dev/null 2> $OUT/pmc_fetch.err || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --config $CFG $NA --steps 1 --warmup 0 --no-cpu --sustain-s 0 > /dev/null 2> $OUT/pmc_write.err || exit 3
python tools/summarize_prof.py $OUT > $OUT/summary.json || exit 4
echo done
