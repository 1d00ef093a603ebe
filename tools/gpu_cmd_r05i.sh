set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 200 python3 bench.py --config c3 --no-cpu --steps 200 --warmup 20 > gpurun_out/r05i/c3.json 2> gpurun_out/r05i/c3.err || { tail -5 gpurun_out/r05i/c3.err; exit 1; }
cat gpurun_out/r05i/c3.err | grep -v amdgpu.ids | head -5
python3 -c "import json; d=json.load(open('gpurun_out/r05i/c3.json')); print(d['value']/1e6)"
