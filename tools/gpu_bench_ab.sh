# Interleaved A/B of bench lines over environment settings (one process per setting and round).
#   tools/gpu_bench_ab.sh TAG ROUNDS "BENCH ARGS" "VAR=a" "VAR=b" ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; R=${2:-3}; A=$3; shift 3
mkdir -p $O
i=0
for rep in $(seq 1 $R); do
  for s in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 env $s python3 bench.py $A > $O/b_$i.json 2> $O/b_$i.err || { tail -5 $O/b_$i.err; exit 1; }
    python3 - "$s" $O/b_$i.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1]); r = d["roofline"]
print(f"{sys.argv[1]:40s} value {d['value']/1e6:8.3f} M/s  ms/step {d['ms_per_step']:.3f}  stage {r['per_launch']['avg_ms']:.3f} ms  frac {r['frac']:.4f}", flush=True)
PY
  done
done
