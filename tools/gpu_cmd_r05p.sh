set -o pipefail
for t in 1 8 16 24; do echo "== host_prof threads $t"; BCC_PREPARE_TRACE=1 BCC_HOST_THREADS=$t timeout -k 10 100 ./host_prof_box 1000000 2>&1 | grep -E "prepare n=|cpu " | tail -3; done
run() { timeout -k 10 150 env "$@" python3 tools/dropin_e2e.py 1000000 10 2>&1 | grep -v amdgpu.ids; }
run BCC_HOST_THREADS=16 && run BCC_HOST_THREADS=24 && run BCC_HOST_THREADS=32 && run BCC_HOST_THREADS=48
