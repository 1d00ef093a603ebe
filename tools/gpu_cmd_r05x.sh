set -o pipefail
timeout -k 10 300 python3 -u -m pytest tests/test_taproot_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05x_tests.log 2>&1 || { tail -30 gpurun_out/r05x_tests.log; exit 1; }
tail -2 gpurun_out/r05x_tests.log
for r in 131072 65536 262144; do
BCC_TAPROOT_ROUND=$r timeout -k 10 120 python3 tools/e2e_timeline.py c5t 8 2>&1 | grep -E "ms per call" | sed "s/^/round $r: /"
done
