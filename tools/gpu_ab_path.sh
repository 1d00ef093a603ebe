#!/bin/bash
# GPU: full -m gpu suite on the default (square-root-free) ECDSA path, then interleaved C2 / C4
# benches of the twist path against the round-1 path (BCC_ECDSA_PATH=legacy) on one box.
# usage: tools/gpu_ab_path.sh TAG [ROUNDS]
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
R=${2:-2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for i in $(seq 1 $R); do
  for p in twist legacy; do
    env=""; [ $p = legacy ] && env="BCC_ECDSA_PATH=legacy"
    env $env timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 > $O/c2_${p}_$i.json 2> $O/c2_${p}_$i.err || { tail -20 $O/c2_${p}_$i.err; exit 2; }
  done
done
for p in twist legacy; do
  env=""; [ $p = legacy ] && env="BCC_ECDSA_PATH=legacy"
  env $env timeout -k 10 300 python bench.py --config c4 --no-cpu > $O/c4_${p}.json 2> $O/c4_${p}.err || { tail -20 $O/c4_${p}.err; exit 3; }
done
python3 - "$O" <<'PY'
import glob, json, os, sys
O = sys.argv[1]
for f in sorted(glob.glob(f"{O}/c*_*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), round(d["value"] / 1e6, 2), d["unit"], "ms", round(d["ms_per_step"], 3),
          "frac", round(d["roofline"]["frac"], 4), "valid", d.get("verdicts_valid"),
          "e2e", (d.get("drop_in_end_to_end") or {}).get("inputs_per_s"))
PY
