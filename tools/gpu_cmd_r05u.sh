set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
echo "== c3_stage_pmc (no profiler)"
timeout -k 5 60 python3 -X faulthandler tools/c3_stage_pmc.py 3 > $O/c3stage.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $O/c3stage.log | tail -30
