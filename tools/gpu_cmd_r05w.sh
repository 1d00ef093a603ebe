set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05w; mkdir -p $O
cd /tmp
BCC_TAPROOT_ROUND=${ROUND:-131072} BCC_TAPROOT_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o run -- python3 $GRAFT_REPO_ROOT/tools/e2e_timeline.py c5t 4 > $O/run.log 2>&1 || { tail $O/run.log; exit 2; }
grep "ms per call" $O/run.log
