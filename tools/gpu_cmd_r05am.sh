set -o pipefail
for a in "--steps 1 --warmup 0 --sustain-s 0" "--steps 10 --warmup 2 --sustain-s 0" "--steps 10 --warmup 2"; do
timeout -k 10 400 python bench.py --config c4 --no-cpu $a > gpurun_out/r05am.json 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r05am.json')); print('$a', d['drop_in_end_to_end']['calls_ms'])"
done
