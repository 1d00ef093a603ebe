set -o pipefail
run() { timeout -k 10 120 env "$@" python3 tools/tuple_e2e.py 8000000 4 2>&1 | grep -v amdgpu.ids; }
for rep in 1 2; do
run BCC_TUPLE_SLOTS=2 && run BCC_TUPLE_SLOTS=3 && run BCC_TUPLE_SLOTS=3 BCC_TUPLE_ROUND=1048576 && run BCC_TUPLE_SLOTS=3 BCC_TUPLE_ROUND=4194304
done
