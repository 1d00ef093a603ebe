#!/bin/bash
# C3 on the current tree: three bench lines (no CPU baseline) and one kernel + copy trace.
O=gpurun_out/${1:-c3probe}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --config c3 --no-cpu --steps 200 --warmup 20 > $O/bench_c3_$i.json 2> $O/bench_c3_$i.err || { tail -5 $O/bench_c3_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_c3_$i.json')); b=d['batch_stats']; print('c3', $i, round(d['value']/1e6,3), round(d['ms_per_step'],3), 'host', round(b['host_seconds']*1e3,3), 'gpu', round(b['gpu_seconds']*1e3,3), 'interp', round(b['interpret_seconds']*1e3,3), 'prep', round(b['prepare_seconds']*1e3,3), 'hostjobs', round(b['host_jobs_seconds']*1e3,3))"
done
bash tools/c3_copy_trace.sh ${1:-c3probe}/copy && python3 tools/copy_timeline.py $O/copy/trace > $O/copy_timeline.txt 2>&1; head -30 $O/copy_timeline.txt
