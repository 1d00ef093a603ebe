#!/bin/bash
# Round-4 evidence pass on the current tree (run via gpurun): checks, the PMC decomposition of the
# C2 kernels (SQ passes + trace), FETCH / WRITE passes, and the C3 / C5 / C5T bench lines.
# usage: tools/gpu_r04_prof.sh TAG
export TMPDIR=/tmp
T=${1:-r04prof}
O=gpurun_out/$T
mkdir -p $O
bash tools/gpu_check.sh $T || exit 1
bash tools/isa/pmc_decomp.sh $T/isa > $O/isa.log 2>&1 || { tail -20 $O/isa.log; exit 2; }
FULL=1 bash tools/profile_c2.sh $T/prof > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 3; }
tail -15 $O/prof.log
for c in c3 c5 c5t; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', d['value']/1e6, d['ms_per_step'], d['roofline']['frac'])"
done
