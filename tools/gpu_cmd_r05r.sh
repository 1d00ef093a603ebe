set -o pipefail
run() { timeout -k 10 150 env "$@" python3 tools/dropin_e2e.py 1000000 20 2>&1 | grep -v amdgpu.ids; }
for rep in 1 2 3; do for t in 16 24 32 48; do run BCC_HOST_THREADS=$t || exit 1; done; done
