set -o pipefail
run() { timeout -k 10 150 env "$@" python3 tools/dropin_e2e.py 1000000 10 2>&1 | grep -v amdgpu.ids; }
run DUMP=1 BCC_HOST_THREADS=24 && run DUMP=1 BCC_HOST_THREADS=48 && run DUMP=1 BCC_HOST_THREADS=16 && BCC_HOST_THREADS=1 timeout -k 10 100 ./host_prof_box 1000000
