#!/bin/bash
# Interleaved same-box A/B of environment settings on one bench config (run via gpurun).
# usage: tools/gpu_env_ab.sh TAG CONFIG ROUNDS "ENV_A" "ENV_B" ...   ("-" = no env)
export TMPDIR=/tmp
O=gpurun_out/$1; C=$2; R=$3; shift 3
mkdir -p $O
for i in $(seq 1 $R); do
  k=0
  for e in "$@"; do
    k=$((k+1)); v="$e"; [ "$v" = "-" ] && v=""
    env $v timeout -k 10 300 python3 bench.py --config $C --no-cpu --no-extra --steps 10 --warmup 3 --sustain-s 0 > $O/${C}_${k}_$i.json 2> $O/${C}_${k}_$i.err || { tail -20 $O/${C}_${k}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${C}_${k}_$i.json')); print('$C', '[$e]', $i, round(d['value']/1e6,3), d['unit'], round(d['ms_per_step'],3), 'ms')"
  done
done
