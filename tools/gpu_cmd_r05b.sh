set -o pipefail
mkdir -p gpurun_out
cp abvar/v5/librbc_amd.so abvar/v5/librbc_bench.so rust-bitcoinconsensus_amd/
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_field_gpu.py > gpurun_out/field_v5.log 2>&1 || { tail -30 gpurun_out/field_v5.log; exit 1; }
tail -2 gpurun_out/field_v5.log
bash tools/ab_prim.sh 2 c2 v4 v5 v5x 2>&1 | tee gpurun_out/ab_v5_c2.txt
for i in 1 2; do for v in v4 v5 v5x; do
  cp abvar/$v/librbc_amd.so abvar/$v/librbc_bench.so rust-bitcoinconsensus_amd/
  timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/ab/${v}_c5_$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_c5_$i.json')); print('$v c5 $i', round(d['value']/1e6,2), round(d['roofline']['frac'],4))" | tee -a gpurun_out/ab_v5_c5.txt
done; done
