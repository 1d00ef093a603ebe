#!/bin/bash
# One GPU call's standard checks: the -m gpu suite, smoke(), the default bench line.
# usage: tools/gpu_check.sh TAG [extra bench args]   (outputs under gpurun_out/TAG)
export TMPDIR=/tmp
O=gpurun_out/${1:-check}; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e6, d['ms_per_step'], d['roofline']['frac'])"
