set -o pipefail
mkdir -p gpurun_out/r05f
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_block_gpu.py tests/test_consensus_gpu.py > gpurun_out/r05f/pytest.log 2>&1 || { grep -v "^  File" gpurun_out/r05f/pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/r05f/pytest.log
bash tools/gpu_c3_ab_env.sh r05f/ab 3 "BCC_SHARDS_PER_WORKER=1" "BCC_SHARDS_PER_WORKER=2" "BCC_SHARDS_PER_WORKER=4" "BCC_SHARDS_PER_WORKER=4 BCC_EARLY_Q=0"
