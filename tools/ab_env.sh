#!/bin/bash
# Interleaved A/B of environment settings on one bench config (run on the GPU box via gpurun):
#   bash tools/ab_env.sh TAG ROUNDS CONFIG "VAR=1 OTHER=2" "VAR=0" ...   (use "-" for no setting)
# -> gpurun_out/TAG/ab_<config>_<k>_<round>.json, one summary line per run.
T=$1; R=$2; C=$3; shift 3
O=gpurun_out/$T
mkdir -p $O
for i in $(seq 1 $R); do
  k=0
  for e in "$@"; do
    k=$((k+1)); [ "$e" = "-" ] && e=""
    f=$O/ab_${C}_${k}_$i
    env $e timeout -k 10 300 python bench.py --config $C --steps 20 --warmup 10 --no-cpu > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 -c "import json; d=json.load(open('$f.json')); r=d['roofline']; b=d.get('batch_stats',{}); print('$C', '[$e]', $i, round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],3), 'stage', round(r.get('per_launch',{}).get('avg_ms',0),3), 'frac', round(r['frac'],4), 'valid', d['verdicts_valid'], 'gpu_ms', round(1e3*b.get('gpu_seconds',0),3), 'host_ms', round(1e3*b.get('host_seconds',0),3))"
  done
done
