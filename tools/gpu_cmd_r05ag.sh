set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests/test_block_gpu.py tests/test_sharding_gpu.py tests/test_consensus_gpu.py tests/test_workload_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ag_tests.log 2>&1 || { tail -30 gpurun_out/r05ag_tests.log; exit 1; }
tail -2 gpurun_out/r05ag_tests.log
run() { timeout -k 10 200 env "$@" python3 bench.py --config c3 --no-cpu --no-extra --steps 300 --warmup 30 2>/dev/null | python3 -c "import json,sys; print('$*', round(json.load(sys.stdin)['value']/1e6,3))"; }
for rep in 1 2 3; do run BCC_EARLY_SIGHASH=0 || exit 1; run BCC_EARLY_SIGHASH=1 || exit 1; done
