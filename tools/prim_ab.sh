#!/bin/bash
# Primitive cycles (mi_primbench) of library variants, interleaved: bash tools/prim_ab.sh ROUNDS NAME...
R=$1; shift
D=rust-bitcoinconsensus_amd
cp $D/librbc_amd.so /tmp/head_amd.so; cp $D/librbc_bench.so /tmp/head_bench.so
for i in $(seq 1 $R); do for v in "$@"; do
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
print('$v', $i, ', '.join(out))
" || exit 1
done; done
cp /tmp/head_amd.so $D/librbc_amd.so; cp /tmp/head_bench.so $D/librbc_bench.so
