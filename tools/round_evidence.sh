#!/bin/bash
# Round evidence on the current build (run via gpurun): C2 rocprof trace + SQ / FETCH / WRITE
# passes, then the default bench line (with the CPU baseline) and the C3 / C4 / C5 / C5T lines,
# then the drop-in end to end with cgroup accounting, best of 3 and 20 calls back to back.
# usage: tools/round_evidence.sh TAG
export TMPDIR=/tmp
T=${1:-r02x}
O=gpurun_out/$T
mkdir -p $O
FULL=1 bash tools/profile_c2.sh $T > $O/profile.txt 2>&1 || { tail -20 $O/profile.txt; exit 1; }
tail -14 $O/profile.txt
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 2; }
for c in c3 c4 c5 c5t; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 3; }
done
python3 - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for f in ("c2", "c3", "c4", "c5", "c5t"):
    d = json.load(open(f"{O}/bench_{f}.json"))
    cb = d.get("cpu_baseline") or {}
    print(f, round(d["value"] / 1e6, 2), d["unit"], "ms", round(d["ms_per_step"], 3), "frac",
          round(d["roofline"]["frac"], 4), "cpu", cb.get("value"), "mism", cb.get("gpu_verdict_mismatches"),
          "e2e", (d.get("drop_in_end_to_end") or {}).get("inputs_per_s"))
PY
timeout -k 10 200 python -u tools/e2e_cgroup.py 1000000 0:0 > $O/e2e.txt 2>&1 || { tail -5 $O/e2e.txt; exit 4; }
grep best_ms $O/e2e.txt
timeout -k 10 200 python -u tools/e2e_sustained.py 1000000 20 0 > $O/e2e_sustained.txt 2>&1 || { tail -5 $O/e2e_sustained.txt; exit 5; }
cat $O/e2e_sustained.txt
