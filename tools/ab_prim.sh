#!/bin/bash
# Interleaved A/B of library variants (tools/abvar_both.sh): the field / group primitives
# (mi_primbench: SIMD cycles per primitive per wave) and the C2 bench line, per round and variant.
#   bash tools/ab_prim.sh ROUNDS CONFIG NAME...   -> gpurun_out/ab/<NAME>_<CONFIG>_<i>.json
R=$1; C=$2; shift 2
mkdir -p gpurun_out/ab
D=rust-bitcoinconsensus_amd
cp $D/librbc_amd.so /tmp/head_amd.so; cp $D/librbc_bench.so /tmp/head_bench.so
for i in $(seq 1 $R); do
  for v in "$@"; do
    cp abvar/$v/librbc_amd.so abvar/$v/librbc_bench.so $D/ || exit 1
    timeout -k 10 120 python3 -c "
import ctypes, sys
sys.path.insert(0, '$D')
from bitcoinconsensus_amd import blib
L = blib()
names = ['fe_mul', 'fe_sqr', 'fe_add', 'fe_sub', 'fe_shl1', 'gej_double', 'gej_add_mixed']
out = []
for p in range(7):
    cyc = ctypes.c_double(); ms = ctypes.c_double()
    assert L.mi_primbench(p, 4000 if p < 5 else 400, 2, ctypes.byref(cyc), ctypes.byref(ms)) == 0
    out.append('%s %.1f' % (names[p], cyc.value))
print('$v', $i, 'prim cycles/wave:', ', '.join(out))
" || exit 1
    timeout -k 10 200 python3 bench.py --config $C --steps 20 --warmup 10 --no-cpu > gpurun_out/ab/${v}_${C}_$i.json 2> gpurun_out/ab/${v}_${C}_$i.err || { tail -5 gpurun_out/ab/${v}_${C}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_${C}_$i.json')); print('$v', '$C', $i, round(d['value']/1e6,2), round(d['ms_per_step'],3), round(d['roofline']['per_launch']['avg_ms'],3), round(d['roofline']['frac'],4), d.get('verdicts_valid'))"
  done
done
cp /tmp/head_amd.so $D/librbc_amd.so; cp /tmp/head_bench.so $D/librbc_bench.so
