#!/bin/bash
# PMC passes over one 262,144-input bench step (run via gpurun): SQ issue/wait breakdown,
# instruction-cache behaviour and the effective clock, per kernel.
export TMPDIR=/tmp
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
grep -o -E "SQC?_[A-Z_]*ICACHE[A-Z_]*|SQ_INST_CYCLES[A-Z_]*|SQ_ACTIVE_INST_[A-Z]*|GRBM_GUI_ACTIVE" $OUT/counters_list.txt | sort -u > $OUT/counters_interesting.txt
B="python bench.py --n 262144 --steps 1 --warmup 0 --no-cpu"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $OUT/sq -o run --output-format csv -- $B > /dev/null 2> $OUT/sq.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE -d $OUT/ic -o run --output-format csv -- $B > /dev/null 2> $OUT/ic.err || exit 2
for f in $(find $OUT/sq $OUT/ic -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", "")[:40]
    agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(agg.items()):
    if "ladder" in k or "prep" in k or "sinv" in k:
        print(f"{k:42s} {c:28s} {v:.4g}")
PY
done
