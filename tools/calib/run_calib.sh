#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/calib/fetch_calib (run via gpurun).
# usage: tools/calib/run_calib.sh TAG   -> gpurun_out/TAG/{fetch,write}/..., summary.txt
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-calib}
mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/calib/fetch_calib > $O/calib.txt 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/calib/fetch_calib > /dev/null 2> $O/write.err || { tail -5 $O/write.err; exit 2; }
cd $GRAFT_REPO_ROOT
python3 - $O <<'PY' | tee $O/summary.txt
import csv, glob, sys, collections
O = sys.argv[1]
print(open(O + "/calib.txt").read().strip())
for kind in ("fetch", "write"):
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{O}/{kind}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]] += float(r["Counter_Value"])
    for k, v in agg.items():
        print(f"{kind:5s} {k:40s} {v * 1024:.4g} bytes")
PY
