#!/bin/bash
# e2e pipeline A/B at several host thread counts (BCC_HOST_THREADS is read once per process)
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
mkdir -p $O
nproc > $O/cpuinfo.txt; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))" >> $O/cpuinfo.txt
cat /sys/fs/cgroup/cpu.max >> $O/cpuinfo.txt 2>/dev/null
cat $O/cpuinfo.txt
for t in 16 12 8; do
  BCC_HOST_THREADS=$t timeout -k 10 200 python -u tools/e2e_ab.py 1000000 0 262144 > $O/e2e_t$t.txt 2>&1 || { tail -5 $O/e2e_t$t.txt; exit 2; }
  echo "threads $t"; tail -2 $O/e2e_t$t.txt
done
