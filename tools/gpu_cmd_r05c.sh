set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_block_gpu.py tests/test_sighash_goldens.py > gpurun_out/r05c/pytest.log 2>&1 || { tail -30 gpurun_out/r05c/pytest.log; exit 1; }
tail -2 gpurun_out/r05c/pytest.log
bash tools/gpu_c3_sweep.sh r05c/sweep 0 100 160 220
bash tools/c3_copy_trace.sh r05c/copy && python3 tools/copy_timeline.py gpurun_out/r05c/copy/trace > gpurun_out/r05c/copy_timeline.txt 2>&1; head -20 gpurun_out/r05c/copy_timeline.txt
