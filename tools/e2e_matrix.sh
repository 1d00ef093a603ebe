#!/bin/bash
# e2e verify_batch probe matrix: pipeline chunk sizes (run on the GPU box)
echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
for c in ${CHUNKS:-0 250000 500000}; do
  echo "== BCC_PIPELINE_CHUNK=$c $*"
  env BCC_PIPELINE_CHUNK=$c "$@" timeout -k 10 200 python tools/e2e_probe.py 1000000 2>&1 | grep items || exit 1
done
