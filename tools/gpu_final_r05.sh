# Round-5 final evidence on the current tree: pytest -m gpu, smoke(), one bench line per config.
set -o pipefail
O=gpurun_out/${1:-r05_final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for c in c2 c3 c4 c5 c5t; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$c.json'))
e=d.get('drop_in_end_to_end') or {}
print('$c', round(d['value']/1e6,2), d['unit'], 'frac', round(d['roofline']['frac'],3), 'traffic', d['roofline'].get('traffic'), 'cpu', round((d.get('cpu_baseline') or {}).get('value',0)), 'e2e', {k: (round(v,3) if isinstance(v,float) else v) for k,v in e.items() if k!='entry'})"
done
