#!/bin/bash
# Round-end evidence on the current tree (run via gpurun): -m gpu suite + smoke + C2 bench, the
# C3 / C4 / C5 / C5T bench lines, then the >=10M agreement legs.  usage: tools/gpu_final.sh TAG
export TMPDIR=/tmp
T=${1:-final}
O=gpurun_out/$T
mkdir -p $O
bash tools/gpu_check.sh $T || exit 1
for c in c3 c4 c5 c5t; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 2; }
  python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', d['value']/1e6, d['ms_per_step'], d['roofline']['frac'], d.get('gpu_vs_cpu'))"
done
bash tools/gpu_agree_all.sh ${T}_agree || exit 3
