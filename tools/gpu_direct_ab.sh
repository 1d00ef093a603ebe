# Direct upload (bcc_set_direct_upload) on the GPU box: the GPU suite, then the drop-in with the
# switch alternating call by call in one process (tools/dropin_interleave.py), then one C2 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-direct}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 tools/dropin_interleave.py 1000000 12 500000:0:1:1:0 500000:0:1:1:1 > $O/interleave_$r.txt 2>&1 || { tail -20 $O/interleave_$r.txt; exit 2; }
  cat $O/interleave_$r.txt
done
timeout -k 10 600 python bench.py --no-side > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 3; }
python3 tools/bench_summary.py $O/bench_c2.json
