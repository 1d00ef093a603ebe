#!/bin/bash
# Stall breakdown of the signature kernels (run via gpurun): two SQ counter passes over one C2 step.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-stall}
mkdir -p $OUT
B="python bench.py --steps 1 --warmup 0 --no-cpu"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_IFETCH SQ_IFETCH_LEVEL -d $OUT/p1 -o run --output-format csv -- $B > /dev/null 2> $OUT/p1.err || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- $B > /dev/null 2> $OUT/p2.err || exit 2
for f in $(find $OUT/p1 $OUT/p2 -name "*counter_collection.csv"); do python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", "").split("(")[0].replace("bcc::", "")
    if not any(x in k for x in ("ladder", "prep", "key", "sinv")): continue
    agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
    print(f"{k:30s} {c:26s} {v:.4g}")
PY
done
