set -o pipefail
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05y_tests.log 2>&1 || { tail -30 gpurun_out/r05y_tests.log; exit 1; }
tail -2 gpurun_out/r05y_tests.log
for r in 131072 262144; do
BCC_TAPROOT_ROUND=$r timeout -k 10 120 python3 tools/e2e_timeline.py c5t 8 2>&1 | grep -E "ms per call" | sed "s/^/round $r: /"
done
timeout -k 10 120 python3 tools/tuple_e2e.py 8000000 4 2>&1 | grep -v amdgpu.ids
run() { timeout -k 10 150 env "$@" python3 tools/dropin_e2e.py 1000000 20 2>&1 | grep -v amdgpu.ids; }
run BCC_X=1 && run BCC_X=2
for i in 1 2; do timeout -k 10 200 python3 bench.py --config c3 --no-cpu --no-extra --steps 200 --warmup 20 2>/dev/null | python3 -c "import json,sys; print('c3', json.load(sys.stdin)['value']/1e6)"; done
