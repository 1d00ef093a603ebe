set -o pipefail
run() { timeout -k 10 150 env "$@" python3 tools/dropin_e2e.py 1000000 10 2>&1 | grep -v amdgpu.ids; }
run BCC_X=0 && run BCC_HOST_THREADS=16 && run BCC_HOST_THREADS=24 && run BCC_HOST_THREADS=32 && run BCC_HOST_THREADS=48 && run BCC_HOST_THREADS=16 BCC_PIPELINE_CHUNK=250000 && run BCC_HOST_THREADS=24 BCC_PIPELINE_CHUNK=250000
