#!/bin/bash
# Default host threads = 3 x the cgroup quota (run via gpurun): GPU suite, sustained drop-in at the
# default against 16 threads, C3 / C5T / C2 bench lines at the default against BCC_HOST_THREADS=16.
export TMPDIR=/tmp
T=${1:-r03t}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u tools/e2e_sustained.py 1000000 20 0 16 > $O/sustained.txt 2>&1 || { tail -5 $O/sustained.txt; exit 2; }
cat $O/sustained.txt
cp rust-bitcoinconsensus_amd/librbc_amd.so abvar/head/librbc_amd.so
for c in c3 c5t; do bash tools/ab_run.sh 2 $c head head@BCC_HOST_THREADS=16 || exit 3; done
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print(round(d['value']/1e6,2), d['drop_in_end_to_end'])"
