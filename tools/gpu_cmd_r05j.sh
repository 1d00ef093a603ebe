set -o pipefail
mkdir -p gpurun_out/r05j
timeout -k 10 500 python3 -u -m pytest tests/test_tuples_gpu.py tests/test_sharding_gpu.py tests/test_block_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05j/tests.log 2>&1 || { tail -40 gpurun_out/r05j/tests.log; exit 1; }
tail -3 gpurun_out/r05j/tests.log
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --steps 10 --warmup 2 > gpurun_out/r05j/c4.json 2> gpurun_out/r05j/c4.err || { tail -5 gpurun_out/r05j/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05j/c4.json')); print(d['value']/1e6, d['drop_in_end_to_end'])"
for i in 1 2; do
timeout -k 10 200 python3 bench.py --config c3 --no-cpu --steps 200 --warmup 20 > gpurun_out/r05j/c3_$i.json 2> gpurun_out/r05j/c3_$i.err || { tail -5 gpurun_out/r05j/c3_$i.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r05j/c3_$i.err | head -5 || true
python3 -c "import json; d=json.load(open('gpurun_out/r05j/c3_$i.json')); print(d['value']/1e6)"
done
