set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05aa; mkdir -p $O
cd /tmp
BCC_TUPLE_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o run -- python3 $GRAFT_REPO_ROOT/tools/tuple_e2e.py 8000000 3 > $O/run.log 2>&1 || { tail $O/run.log; exit 2; }
grep "M/s" $O/run.log
