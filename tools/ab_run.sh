#!/bin/bash
# Interleaved A/B of library variants with optional env per entry, run on the GPU box via gpurun:
#   [BENCH_ARGS=...] bash tools/ab_run.sh ROUNDS CONFIG NAME[@ENV=VAL] ...   -> gpurun_out/ab/<entry>_i.json
R=$1; C=$2; shift 2
mkdir -p gpurun_out/ab
cp rust-bitcoinconsensus_amd/librbc_amd.so /tmp/librbc_amd_head.so
for i in $(seq 1 $R); do
  for e in "$@"; do
    v=${e%%@*}; env=""; [ "$v" != "$e" ] && env=${e#*@}
    tag=$(echo "$e" | tr '@=/ ' '____')
    cp abvar/$v/librbc_amd.so rust-bitcoinconsensus_amd/librbc_amd.so || exit 1
    env $env timeout -k 10 200 python bench.py --config $C ${BENCH_ARGS:---steps 20 --warmup 10 --no-cpu} > gpurun_out/ab/${tag}_${C}_$i.json 2> gpurun_out/ab/${tag}_${C}_$i.err || { tail -5 gpurun_out/ab/${tag}_${C}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${tag}_${C}_$i.json')); print('$tag', '$C', $i, round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['roofline']['per_launch']['avg_ms'],3), round(d['roofline']['frac'],4), d['verdicts_valid'])"
  done
done
cp /tmp/librbc_amd_head.so rust-bitcoinconsensus_amd/librbc_amd.so
