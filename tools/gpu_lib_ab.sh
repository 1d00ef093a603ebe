# Drop-in A/B of library builds in alternating processes (abvar/<NAME>/librbc_amd.so swapped in):
#   tools/gpu_lib_ab.sh TAG ROUNDS NAME...   -> gpurun_out/TAG/dropin.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; R=$2; shift 2
mkdir -p $O
cp rust-bitcoinconsensus_amd/librbc_amd.so /tmp/librbc_amd_head.so
for i in $(seq 1 $R); do
  for v in "$@"; do
    cp abvar/$v/librbc_amd.so rust-bitcoinconsensus_amd/librbc_amd.so || exit 1
    printf "%s %s: " $v $i >> $O/dropin.txt
    PHASES=1 timeout -k 10 200 python3 tools/dropin_e2e.py 1000000 20 >> $O/dropin.txt 2>&1 || { cp /tmp/librbc_amd_head.so rust-bitcoinconsensus_amd/librbc_amd.so; tail -5 $O/dropin.txt; exit 1; }
  done
done
cp /tmp/librbc_amd_head.so rust-bitcoinconsensus_amd/librbc_amd.so
cat $O/dropin.txt
