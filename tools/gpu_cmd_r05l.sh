set -o pipefail
mkdir -p gpurun_out/r05l
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BCC_TUPLE_TRACE=1 BCC_TUPLE_ROUND=2097152 BCC_TUPLE_FIRST=262144 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/r05l/prof -o tl -- python3 tools/tuple_e2e.py 8000000 2 > gpurun_out/r05l/run.log 2>&1 || { tail -20 gpurun_out/r05l/run.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05l/run.log | grep "bcc\|M/s" | tail -4
find gpurun_out/r05l/prof -name "*.csv" | head
