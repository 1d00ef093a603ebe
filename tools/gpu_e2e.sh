#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/e2e_ab.py 1000000 0 131072 262144 524288 > $O/e2e_ab.txt 2>&1 || { tail -20 $O/e2e_ab.txt; exit 2; }
tail -4 $O/e2e_ab.txt
timeout -k 10 300 python bench.py --config c3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', round(d['value']/1e6,3), d['ms_per_step'])"
