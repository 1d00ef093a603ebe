#!/bin/bash
mkdir -p gpurun_out/c3ab
for i in 1 2; do
for e in "X=1" "BCC_ECDSA_PATH=legacy" "BCC_OVERLAP_RUNS=0"; do
  env $e timeout -k 10 200 python bench.py --config c3 --no-cpu > gpurun_out/c3ab/$e.$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c3ab/$e.$i.json')); b=d.get('batch_stats',{}); print('$e', $i, round(d['value']/1e6,3), round(d['ms_per_step'],3), 'gpu', round(1e3*b.get('gpu_seconds',0),2), 'host', round(1e3*b.get('host_seconds',0),2))"
done; done
timeout -k 10 300 python bench.py --no-cpu --steps 10 > gpurun_out/c3ab/c2.json 2>/dev/null && python3 -c "import json; d=json.load(open('gpurun_out/c3ab/c2.json')); print('c2', round(d['value']/1e6,2), round(d['roofline']['frac'],4))"
