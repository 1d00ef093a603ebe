set -o pipefail
timeout -k 10 400 python bench.py --config c4 --no-cpu > gpurun_out/r05aj_c4.json 2> gpurun_out/r05aj_c4.err || { tail -20 gpurun_out/r05aj_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r05aj_c4.json')); print(d['value']/1e6, d['drop_in_end_to_end'])"
timeout -k 10 120 python3 tools/tuple_e2e.py 8000000 4 2>&1 | grep -v amdgpu.ids
