#!/bin/bash
# Device key-hash check (BCC_DEVICE_KEY_HASH) on the GPU box: the GPU suite, then interleaved A/B of
# the drop-in end to end and of the C2 / C3 bench lines (run via gpurun).
export TMPDIR=/tmp
T=${1:-r03q}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/gpu_e2e_ab.sh $T 3 "-" "BCC_DEVICE_KEY_HASH=0" || exit 2
bash tools/ab_run.sh 2 c2 head head@BCC_DEVICE_KEY_HASH=0 || exit 3
bash tools/ab_run.sh 2 c3 head head@BCC_DEVICE_KEY_HASH=0 || exit 4
