#!/bin/bash
# The round-end GPU tiers on the current tree: pytest -m gpu, smoke(), one default bench line.
#   bash tools/gpu_suite.sh TAG   -> gpurun_out/TAG/{pytest_gpu.log,smoke.log,bench.json}
T=${1:-suite}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e6, d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
