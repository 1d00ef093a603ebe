#!/bin/bash
# >=10M agreement on the current kernels: 10M C4 tuples + 8M BIP340 rows (GPU vs reference on every
# input), 10M script-level items through verify_batch, and the C3 bench line.  usage: TAG
export TMPDIR=/tmp
O=gpurun_out/${1:-r02x}
mkdir -p $O
timeout -k 10 900 python -u tools/agreement.py --c4 10000000 --c5 8000000 --out $O/agreement_c4_10M_c5_8M.json > $O/agreement_c4_c5.log 2>&1 || { tail -30 $O/agreement_c4_c5.log; exit 1; }
tail -3 $O/agreement_c4_c5.log
timeout -k 10 1000 python -u tools/agreement.py --c4 0 --c5 0 --scripts 10000000 --out $O/agreement_scripts_10M.json > $O/agreement_scripts.log 2>&1 || { tail -30 $O/agreement_scripts.log; exit 2; }
tail -3 $O/agreement_scripts.log
timeout -k 10 400 python bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 3; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['value']/1e6, d['unit'], (d.get('cpu_baseline') or {}).get('value'))"
