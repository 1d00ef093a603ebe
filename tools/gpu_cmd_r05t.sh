set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05t; mkdir -p $O
bash tools/gpu_c3_traffic.sh r05_c3traffic || exit 1
cd /tmp
for c in c5t c3; do
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl_$c -o run -- python3 $GRAFT_REPO_ROOT/tools/e2e_timeline.py $c 6 > $O/tl_$c.log 2>&1 || { tail $O/tl_$c.log; exit 2; }
grep "ms per call" $O/tl_$c.log
done
cd $GRAFT_REPO_ROOT
python3 tools/timeline_summary.py $O/tl_c5t 30 > $O/tl_c5t.txt && tail -1 $O/tl_c5t.txt
python3 tools/timeline_summary.py $O/tl_c3 4 > $O/tl_c3.txt && tail -1 $O/tl_c3.txt
