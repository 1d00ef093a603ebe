set -o pipefail
timeout -k 10 120 python3 tools/tuple_e2e.py 8000000 4 2>&1 | grep -v amdgpu.ids
WITH_TORCH=1 timeout -k 10 120 python3 tools/tuple_e2e.py 8000000 4 2>&1 | grep -v amdgpu.ids
