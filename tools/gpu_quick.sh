#!/bin/bash
# GPU: parity tests of the consensus paths + C2/C3 bench + C3 kernel trace.  usage: TAG
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 2; }
timeout -k 10 300 python bench.py --config c3 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 3; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/c3trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --no-cpu --steps 3 --warmup 1 > /dev/null 2> $GRAFT_REPO_ROOT/$O/c3_prof.err || { tail -20 $GRAFT_REPO_ROOT/$O/c3_prof.err; exit 4; }
cd $GRAFT_REPO_ROOT
python3 - "$O" <<'PY'
import json, sys, glob, csv
O = sys.argv[1]
for f in ("c2", "c3"):
    d = json.load(open(f"{O}/bench_{f}.json"))
    print(f, round(d["value"] / 1e6, 2), "ms", round(d["ms_per_step"], 3), "frac", round(d["roofline"]["frac"], 4),
          "sighash", round(d.get("sighash_stage", {}).get("avg_ms", 0), 3), "e2e", d.get("drop_in_end_to_end", {}).get("inputs_per_s") if d.get("drop_in_end_to_end") else None,
          d.get("drop_in_end_to_end", {}).get("host_ms") if d.get("drop_in_end_to_end") else None)
for p in glob.glob(f"{O}/c3trace/*kernel_stats.csv"):
    for row in csv.DictReader(open(p)):
        if "ubench" in row["Name"]: continue
        print(f'{row["Name"][:50]:50s} calls {row["Calls"]:>4s} avg_us {float(row["AverageNs"])/1e3:9.1f}')
PY
