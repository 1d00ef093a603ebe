#!/bin/bash
# Kernel trace of one bench config; prints per-kernel averages.  usage: TAG CONFIG
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
C=${2:-c2}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/${C}trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $C --no-cpu --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$O/${C}_under_prof.json 2> $GRAFT_REPO_ROOT/$O/${C}_prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/${C}_prof.err; exit 4; }
cd $GRAFT_REPO_ROOT
python3 tools/trace_step.py "$O/${C}trace" > "$O/${C}_step_kernels.txt"; cat "$O/${C}_step_kernels.txt"
python3 - "$O/${C}trace" <<'PY'
import sys, glob, csv
for p in glob.glob(f"{sys.argv[1]}/*kernel_stats.csv"):
    for row in csv.DictReader(open(p)):
        if "ubench" in row["Name"]: continue
        print(f'{row["Name"][:50]:50s} calls {row["Calls"]:>4s} avg_us {float(row["AverageNs"])/1e3:9.1f}')
PY
