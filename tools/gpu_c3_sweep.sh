#!/bin/bash
# C3 at several host-chain thresholds (BCC_HOST_CHAIN_BLOCKS), interleaved, 3 rounds.
O=gpurun_out/${1:-c3sweep}
shift
mkdir -p $O
for i in 1 2 3; do for k in "$@"; do
  BCC_HOST_CHAIN_BLOCKS=$k timeout -k 10 200 python3 bench.py --config c3 --no-cpu --steps 300 --warmup 30 > $O/c3_k${k}_$i.json 2> $O/c3_k${k}_$i.err || { tail -5 $O/c3_k${k}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_k${k}_$i.json')); b=d['batch_stats']; print('k=$k', $i, round(d['value']/1e6,3), round(d['ms_per_step'],3), 'host', round(b['host_seconds']*1e3,3), 'gpu', round(b['gpu_seconds']*1e3,3), 'interp', round(b['interpret_seconds']*1e3,3), 'hostjobs', round(b['host_jobs_seconds']*1e3,3), 'hashed', b['host_hashed'])"
done; done
