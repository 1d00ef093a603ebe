#!/bin/bash
# Round 3, GPU pass I: the drop-in's host pass under pipelining (per-worker prepare timing), one
# configuration per process; a C3 kernel trace (timeline of one verify_batch round).
export TMPDIR=/tmp
O=gpurun_out/${1:-r03i}
mkdir -p $O
for c in 0:0 262144:0 0:0; do
  timeout -k 10 200 python -u tools/e2e_cgroup.py 1000000 $c >> $O/e2e.txt 2>&1 || { tail -5 $O/e2e.txt; exit 1; }
done
grep best_ms $O/e2e.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c3trace -o run --output-format csv -- python bench.py --config c3 --steps 3 --warmup 1 --no-cpu > $O/c3_under_trace.json 2> $O/c3trace.err || { tail -5 $O/c3trace.err; exit 2; }
echo done
