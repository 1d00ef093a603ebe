set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_workload_gpu.py tests/test_block_gpu.py tests/test_consensus_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ac_tests.log 2>&1 || { tail -30 gpurun_out/r05ac_tests.log; exit 1; }
tail -2 gpurun_out/r05ac_tests.log
run() { timeout -k 10 150 env "$@" python3 tools/dropin_e2e.py 1000000 20 2>&1 | grep -v amdgpu.ids; }
for rep in 1 2; do
run BCC_CHUNK_LAUNCH_EARLY=0 && run BCC_CHUNK_LAUNCH_EARLY=1 && run BCC_CHUNK_LAUNCH_EARLY=1 BCC_PIPELINE_CHUNK=250000 && run BCC_CHUNK_LAUNCH_EARLY=1 BCC_PIPELINE_CHUNK=340000
done
