set -o pipefail
for rep in 1 2; do for v in 1 0; do
if [ $v = 1 ]; then E="BCC_BENCH_NO_EARLY_ALLOC=1"; else E="BCC_X=0"; fi
timeout -k 10 400 env $E python bench.py --config c2 --no-cpu > gpurun_out/r05ao.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r05ao.json')); e=d['drop_in_end_to_end']; print('$E', round(d['value']/1e6,2), round(e['inputs_per_s']/1e6,2), round(e['sustained_inputs_per_s']/1e6,2), e['sustained_cpu_s_per_M'])"
done; done
