set -o pipefail
mkdir -p gpurun_out/r05g
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_block_gpu.py tests/test_consensus_gpu.py tests/test_ecdsa_tuples_gpu.py tests/test_tuples_gpu.py tests/test_host_verify_gpu.py tests/test_key_hash.py > gpurun_out/r05g/pytest.log 2>&1 || { grep -v "^  File" gpurun_out/r05g/pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/r05g/pytest.log
bash tools/gpu_c3_ab_env.sh r05g/ab 3 "BCC_KEYQ2=0 BCC_EARLY_Q=0" "BCC_KEYQ2=1 BCC_EARLY_Q=0" "BCC_KEYQ2=1 BCC_EARLY_Q=1"
bash tools/c3_copy_trace.sh r05g/copy && python3 tools/copy_timeline.py gpurun_out/r05g/copy/trace > gpurun_out/r05g/copy_timeline.txt 2>&1; head -22 gpurun_out/r05g/copy_timeline.txt
