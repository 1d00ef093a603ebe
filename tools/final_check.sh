#!/bin/bash
# Round-end check on the committed tree (run via gpurun): GPU tests, smoke(), the default bench line.
export TMPDIR=/tmp
O=gpurun_out/${1:-r02final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print(round(d['value']/1e6,2), 'M/s frac', round(r['frac'],4), 'ceiling', r.get('instruction_mix_ceiling',{}).get('frac'), 'cpu', d['cpu_baseline']['value'], 'mism', d['cpu_baseline'].get('gpu_verdict_mismatches'), 'e2e', d['drop_in_end_to_end']['inputs_per_s'])"
