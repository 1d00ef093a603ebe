set -o pipefail
run() { timeout -k 10 150 env "$@" python3 tools/dropin_e2e.py 1000000 20 2>&1 | grep -v amdgpu.ids; }
for rep in 1 2 3 4 5; do
run BCC_CHUNK_LAUNCH_EARLY=0 && run BCC_CHUNK_LAUNCH_EARLY=1
done
