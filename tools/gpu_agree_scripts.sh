#!/bin/bash
# >=10M script-level agreement run (verify_batch vs the reference's verify_script_with_amount).
export TMPDIR=/tmp
mkdir -p gpurun_out/r02d
timeout -k 10 1000 python -u tools/agreement.py --c4 0 --c5 0 --scripts 10000000 --out gpurun_out/r02d/agreement_scripts_10M.json > gpurun_out/r02d/agreement_scripts_10M.log 2>&1 || { tail -30 gpurun_out/r02d/agreement_scripts_10M.log; exit 1; }
tail -4 gpurun_out/r02d/agreement_scripts_10M.log
