#!/bin/bash
# Per-kernel register / scratch / occupancy summary of one HIP source (gfx950).
# usage: tools/kres.sh rust-bitcoinconsensus_amd/csrc/ecdsa_verify.hip
cd "$(dirname "$0")/../rust-bitcoinconsensus_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -c "../$1" \
    -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
    sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' |
    awk '/Function Name/{if(l)print l; l=$3} /VGPRs:|Spill|Occupancy|ScratchSize/{l=l" | "$0} END{print l}'
