#!/bin/bash
# Round 3, GPU pass F: the -m gpu suite, then interleaved A/Bs of this round's switches:
# the split ECDSA ladder (BCC_LADDER_SPLIT) on C2 / C3, the device-built Taproot SigMsg
# (BCC_TAPROOT_HOST_SIGMSG) on C5T, and the drop-in end to end with cgroup accounting.
export TMPDIR=/tmp
O=gpurun_out/${1:-r03f}
T=$(basename $O)
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab_env.sh $T 2 c2 - BCC_LADDER_SPLIT=0 || exit 2
bash tools/ab_env.sh $T 2 c3 - BCC_LADDER_SPLIT=0 || exit 3
bash tools/ab_env.sh $T 2 c5t - BCC_TAPROOT_HOST_SIGMSG=1 || exit 4
timeout -k 10 300 python -u tools/e2e_cgroup.py 1000000 0:0 262144:0 > $O/e2e.txt 2>&1 || { tail -5 $O/e2e.txt; exit 5; }
grep best_ms $O/e2e.txt
