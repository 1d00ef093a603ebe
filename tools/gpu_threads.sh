#!/bin/bash
# Host-thread sweep of the drop-in (run via gpurun): best-of-3 calls per thread count, then
# sustained back-to-back calls with the cgroup's throttling counters.
#   bash tools/gpu_threads.sh TAG "16 32 48 64 96 128" "16 48 64"
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
cfg=""; for t in $2; do cfg="$cfg 0:$t"; done
timeout -k 10 400 python -u tools/e2e_cgroup.py 1000000 $cfg > $O/threads.txt 2>&1 || { tail -5 $O/threads.txt; exit 1; }
grep best_ms $O/threads.txt
timeout -k 10 400 python -u tools/e2e_sustained.py 1000000 20 $3 > $O/sustained.txt 2>&1 || { tail -5 $O/sustained.txt; exit 2; }
cat $O/sustained.txt
