export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02b/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r02b/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r02b/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r02b/bench_c2.json 2> gpurun_out/r02b/bench_c2.err || { tail -20 gpurun_out/r02b/bench_c2.err; exit 2; }
timeout -k 10 300 python bench.py --config c4 --n 2000000 --no-cpu > gpurun_out/r02b/bench_c4.json 2> gpurun_out/r02b/bench_c4.err || { tail -20 gpurun_out/r02b/bench_c4.err; exit 3; }
python3 -c "
import json
for f in ('c2','c4'):
    d=json.load(open(f'gpurun_out/r02b/bench_{f}.json')); print(f, round(d['value']/1e6,2), d['validity_bitmap'], d.get('mismatch_vs_construction'), d['roofline']['frac'])"
