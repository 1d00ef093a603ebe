#!/bin/bash
# Interleaved A/B of library variants (abvar/NAME/librbc_amd.so) on a bench config, run on the GPU
# box via gpurun:  bash tools/ab_run.sh ROUNDS CONFIG NAME1 NAME2 ...
# The box's copy of the tree is scratch, so swapping the in-tree library there is harmless.
R=$1; C=$2; shift 2
mkdir -p gpurun_out/ab
cp rust-bitcoinconsensus_amd/librbc_amd.so /tmp/librbc_amd_head.so
for i in $(seq 1 $R); do
  for v in "$@"; do
    cp abvar/$v/librbc_amd.so rust-bitcoinconsensus_amd/librbc_amd.so || exit 1
    timeout -k 10 200 python bench.py --config $C --steps 10 --warmup 2 --no-cpu > gpurun_out/ab/${v}_${C}_$i.json 2> gpurun_out/ab/${v}_${C}_$i.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/${v}_${C}_$i.json')); print('$v', '$C', $i, round(d['value']/1e6,2), round(d['roofline']['per_launch']['avg_ms'],3), round(d['roofline']['frac'],4))"
  done
done
cp /tmp/librbc_amd_head.so rust-bitcoinconsensus_amd/librbc_amd.so
