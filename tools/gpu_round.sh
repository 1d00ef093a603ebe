#!/bin/bash
# GPU pass (run via gpurun): the full -m gpu suite, smoke(), then the default C2 bench line and
# any extra configs given.  usage: tools/gpu_round.sh TAG [c3 c4 c5 c5t ...]
export TMPDIR=/tmp
T=${1:-r03x}; shift
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 3; }
for c in "$@"; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 4; }
done
python3 - "$O" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.load(open(f)); r = d["roofline"]; cb = d.get("cpu_baseline") or {}
    print(f.split("/")[-1], round(d["value"] / 1e6, 3), d["unit"], "ms", round(d["ms_per_step"], 3),
          "frac", round(r["frac"], 4), "meas", round(r.get("peak_measured", {}).get("frac_vs_measured", 0), 4),
          "clk", round(r.get("peak_measured", {}).get("clock_GHz", 0), 3), "cpu", cb.get("value"),
          "mism", cb.get("gpu_verdict_mismatches"), "e2e", d.get("drop_in_end_to_end"),
          "single", d.get("single_call"), "ref1", cb.get("single_call_us"))
PY
