#!/bin/bash
# Interleaved A/B of two library variants on the C2 bench (run via gpurun):
#   bash tools/ab_c2.sh A B ROUNDS  -> gpurun_out/ab/{A,B}_{i}.json
mkdir -p gpurun_out/ab
for i in $(seq 1 ${3:-3}); do
  for v in $1 $2; do
    cp variants/$v/librbc_amd.so rust-bitcoinconsensus_amd/librbc_amd.so || exit 1
    timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu > gpurun_out/ab/${v}_$i.json 2> gpurun_out/ab/${v}_$i.err || exit 1
  done
done
