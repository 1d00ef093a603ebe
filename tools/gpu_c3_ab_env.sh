#!/bin/bash
# C3 bench lines under several environment settings, interleaved: tools/gpu_c3_ab_env.sh TAG ROUNDS "ENV1" "ENV2" ...
T=$1; R=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for i in $(seq 1 $R); do for e in "$@"; do
  tag=$(echo "$e" | tr ' =' '_-')
  env $e timeout -k 10 200 python3 bench.py --config c3 --no-cpu --steps 300 --warmup 30 > $O/c3_${tag}_$i.json 2> $O/c3_${tag}_$i.err || { tail -5 $O/c3_${tag}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_${tag}_$i.json')); b=d['batch_stats']; print('$e', $i, round(d['value']/1e6,3), round(d['ms_per_step'],3), 'host', round(b['host_seconds']*1e3,3), 'gpu', round(b['gpu_seconds']*1e3,3), 'prep', round(b['prepare_seconds']*1e3,3), 'interp', round(b['interpret_seconds']*1e3,3), 'hostjobs', round(b['host_jobs_seconds']*1e3,3), 'early', b.get('early_rows'), round(b.get('early_seconds',0)*1e3,3))"
done; done
