#!/bin/bash
# C3 (block replay through verify_batch) under env variants, then one kernel trace of the default.
# usage: tools/c3_sweep.sh TAG "ENV1" "ENV2" ...   (each ENV a space-separated VAR=value list or "-")
export TMPDIR=/tmp
O=gpurun_out/${1:-c3sweep}; shift
mkdir -p $O
i=0
for v in "$@"; do
    i=$((i+1))
    if [ "$v" = "-" ]; then v=""; fi
    env $v timeout -k 10 300 python3 bench.py --config c3 --no-cpu --steps 40 --warmup 10 > $O/c3_$i.json 2> $O/c3_$i.err || { tail -20 $O/c3_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_$i.json')); print('$i', '$v', round(d['value']/1e6,3), 'M/s', round(d['ms_per_step'],3), 'ms')"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c3trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --no-cpu --no-extra --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/c3_under_prof.json 2> $GRAFT_REPO_ROOT/$O/c3_prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/c3_prof.err; exit 4; }
cd $GRAFT_REPO_ROOT
python3 tools/round_timeline.py $O/c3trace --rounds 2 > $O/c3_timeline.txt; cat $O/c3_timeline.txt
