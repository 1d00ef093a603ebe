#!/bin/bash
# C3 timeline with host<->device copies: kernel + memory-copy trace of a short C3 bench
# (run via gpurun; no counters).  usage: tools/c3_copy_trace.sh TAG
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-c5tcopy}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5t --no-cpu --no-extra --steps 10 --warmup 3 > $O/c3_under_prof.json 2> $O/c3_prof.err || { tail -20 $O/c3_prof.err; exit 1; }
echo done
