#!/bin/bash
# Interleaved same-box A/B of library variants on the drop-in end-to-end probe (run via gpurun):
#   bash tools/e2e_ab.sh ROUNDS VARIANT ...   (abvar/<VARIANT>/librbc_amd.so)
R=$1; shift
cp rust-bitcoinconsensus_amd/librbc_amd.so /tmp/librbc_amd_head.so
for i in $(seq 1 $R); do
  for v in "$@"; do
    cp abvar/$v/librbc_amd.so rust-bitcoinconsensus_amd/librbc_amd.so || exit 1
    echo "== $v $i"
    timeout -k 10 200 python tools/e2e_probe.py 1000000 2>&1 | grep items || exit 1
  done
done
cp /tmp/librbc_amd_head.so rust-bitcoinconsensus_amd/librbc_amd.so
