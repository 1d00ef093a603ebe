set -o pipefail
mkdir -p gpurun_out/r05k
run() { timeout -k 10 120 env "$@" python3 tools/tuple_e2e.py 8000000 4 2>&1 | grep -v amdgpu.ids; }
run BCC_TUPLE_TRACE=1 && run BCC_TUPLE_TRACE=1 BCC_TUPLE_FIRST=262144 && run BCC_TUPLE_TRACE=1 BCC_TUPLE_ROUND=2097152 BCC_TUPLE_FIRST=262144 && run BCC_TUPLE_TRACE=1 BCC_TUPLE_ROUND=524288 BCC_TUPLE_FIRST=131072
