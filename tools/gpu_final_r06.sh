#!/bin/bash
# Round-6 evidence on the current tree (run via gpurun): pytest -m gpu, smoke(), the default bench
# line and one line per other config, then the rocprofv3 kernel trace + FETCH / WRITE / SQ passes
# of C2, C4 and C5.  usage: tools/gpu_final_r06.sh TAG [noprof]
set -o pipefail
export TMPDIR=/tmp
T=${1:-r06_final}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 3; }
python3 tools/bench_summary.py $O/bench_c2.json
for c in c3 c4 c5 c5t; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
  python3 tools/bench_summary.py $O/bench_$c.json
done
[ "$2" = noprof ] && exit 0
export FULL=1
bash tools/profile_c2.sh ${T}_prof_c2 || exit 5
bash tools/profile_c2.sh ${T}_prof_c4 --config c4 || exit 6
bash tools/profile_c2.sh ${T}_prof_c5 --config c5 || exit 7
