set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 300 python3 -u -m pytest tests/test_sharding_gpu.py tests/test_block_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05i/tests.log 2>&1 || { tail -30 gpurun_out/r05i/tests.log; exit 1; }
tail -3 gpurun_out/r05i/tests.log
for i in 1 2 3; do
timeout -k 10 200 python3 bench.py --config c3 --no-cpu --steps 200 --warmup 20 > gpurun_out/r05i/c3_$i.json 2> gpurun_out/r05i/c3_$i.err || { tail -5 gpurun_out/r05i/c3_$i.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r05i/c3_$i.err | head -5 || true
python3 -c "import json; d=json.load(open('gpurun_out/r05i/c3_$i.json')); print(d['value']/1e6)"
done
