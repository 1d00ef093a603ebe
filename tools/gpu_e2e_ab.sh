#!/bin/bash
# Drop-in end to end A/B of environment settings, one e2e_cgroup process per setting, interleaved
# (run via gpurun):   bash tools/gpu_e2e_ab.sh TAG ROUNDS "VAR=1" "VAR=0" ...   ("-": none)
export TMPDIR=/tmp
T=$1; R=$2; shift 2
O=gpurun_out/$T
mkdir -p $O
for i in $(seq 1 $R); do
  k=0
  for e in "$@"; do
    k=$((k+1)); [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python -u tools/e2e_cgroup.py 1000000 0:0 > $O/e2e_${k}_$i.txt 2>&1 || { tail -5 $O/e2e_${k}_$i.txt; exit 1; }
    echo "[$e] $i $(grep best_ms $O/e2e_${k}_$i.txt)"
  done
done
