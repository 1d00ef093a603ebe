#!/bin/bash
# >=10M agreement on the current tree (north star: 100 % verdict agreement on >= 10M mixed
# inputs), every leg against the REFERENCE (oracle/_ref) on every input:
#   device path  10M C4 tuples + 8M BIP340 rows, 10M script items through verify_batch;
#   host path    10M C4 tuples through bcc_pubkey_verify_batch and 10M script items through
#                verify_batch with every round on the host lane code (the default for lone verify()).
# usage: tools/gpu_agree_all.sh TAG   (outputs under gpurun_out/TAG)
export TMPDIR=/tmp
O=gpurun_out/${1:-agree}
mkdir -p $O
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python -u tools/agreement.py "$@" --out $O/$name.json > $O/$name.log 2>&1 \
        || { tail -30 $O/$name.log; return 1; }
    tail -2 $O/$name.log
}
run device_c4_c5 900 --c4 10000000 --c5 8000000 &&
run device_scripts 1000 --c4 0 --c5 0 --scripts 10000000 &&
run host_c4 900 --c4 0 --c5 0 --host-c4 10000000 &&
run host_scripts 1000 --c4 0 --c5 0 --host-scripts 10000000
