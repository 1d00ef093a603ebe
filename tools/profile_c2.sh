#!/bin/bash
# rocprofv3 evidence for the default C2 bench (run via gpurun): kernel trace, then one SQ VALU
# counter pass (and FETCH / WRITE passes when FULL=1).  usage: TAG [extra bench args]
export TMPDIR=/tmp
T=${1:-r02x}; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O/c2
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-extra --sustain-s 0 $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/c2/trace -o run --output-format csv -- $B --steps 5 --warmup 2 > $O/c2/bench_under_rocprof.json 2> $O/c2_trace.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -d $O/c2/pmc_sq -o run --output-format csv -- $B --steps 1 --warmup 0 > /dev/null 2> $O/c2_sq.err || exit 4
if [ "$FULL" = 1 ]; then
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/c2/pmc_fetch -o run --output-format csv -- $B --steps 1 --warmup 0 > /dev/null 2> $O/c2_fetch.err || exit 2
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/c2/pmc_write -o run --output-format csv -- $B --steps 1 --warmup 0 > /dev/null 2> $O/c2_write.err || exit 3
fi
cd $GRAFT_REPO_ROOT
python3 tools/summarize_prof.py $O/c2 > $O/c2/summary.json || exit 7
python3 - $O <<'PY'
import json, sys
d = json.load(open(sys.argv[1] + "/c2/summary.json"))
for k, e in sorted(d["kernels"].items(), key=lambda x: -x[1].get("total_ns", 0))[:12]:
    p = e.get("pmc_per_launch", {})
    print(f'{k:28s} calls {e.get("calls")} avg_us {e.get("avg_ns", 0)/1e3:9.1f} valu/launch {p.get("SQ_INSTS_VALU", 0):.4g}')
print(d.get("stages"))
PY
