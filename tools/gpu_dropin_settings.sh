# Drop-in settings alternating call by call in one process (tools/dropin_interleave.py), REPS
# processes, then one C2 line:  tools/gpu_dropin_settings.sh TAG REPS SETTING...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; R=${2:-2}; shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  timeout -k 10 300 python3 tools/dropin_interleave.py 1000000 12 "$@" > $O/interleave_$r.txt 2>&1 || { tail -20 $O/interleave_$r.txt; exit 2; }
  cat $O/interleave_$r.txt
done
timeout -k 10 600 python bench.py --no-side > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 3; }
python3 tools/bench_summary.py $O/bench_c2.json
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('sighash bytes', d['sighash_stage']['algorithmic_bytes'])"
