#!/bin/bash
# GPU: full -m gpu suite, then the default C2 bench (no CPU baseline) and the C3 bench.
# usage: tools/gpu_round2.sh TAG
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 2; }
timeout -k 10 300 python bench.py --config c3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 3; }
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for f in ("c2", "c3"):
    d = json.load(open(f"{O}/bench_{f}.json"))
    print(f, round(d["value"] / 1e6, 2), d["unit"], "ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4),
          "sighash", d.get("sighash_stage", {}).get("avg_ms"), "e2e", d.get("drop_in_end_to_end"))
PY
