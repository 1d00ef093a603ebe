#!/bin/bash
# Kernel trace of the C3 bench (per-kernel durations of the sighash stage).
export TMPDIR=/tmp
O=gpurun_out/${1:-r02h}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c3trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --no-cpu --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/c3_prof.json 2> $GRAFT_REPO_ROOT/$O/c3_prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/c3_prof.err; exit 1; }
cd $GRAFT_REPO_ROOT
find $O/c3trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -20
