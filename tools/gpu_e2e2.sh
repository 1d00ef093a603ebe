#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
mkdir -p $O
timeout -k 10 200 python -u tools/e2e_ab.py 1000000 0 262144 524288 > $O/e2e_ab.txt 2>&1 || { tail -5 $O/e2e_ab.txt; exit 2; }
cat $O/e2e_ab.txt
