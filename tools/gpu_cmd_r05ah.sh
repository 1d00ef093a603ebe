set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05ah; mkdir -p $O
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o run -- python3 $GRAFT_REPO_ROOT/tools/e2e_timeline.py c3 8 > $O/run.log 2>&1 || { tail $O/run.log; exit 2; }
grep "ms per call" $O/run.log
cd $GRAFT_REPO_ROOT
python3 tools/timeline_summary.py $O/tl 6 > $O/tl_c3.txt && tail -1 $O/tl_c3.txt
python3 - <<'PY'
import sys
sys.path.insert(0, "rust-bitcoinconsensus_amd")
import bench, bitcoinconsensus_amd as B
job = bench.C3(B, bench.DEFAULT_N["c3"], bench.SEEDS["c3"], 0)
for _ in range(5): job.step(None)
st = B.last_batch_stats()
print({k: round(v*1e3,3) if isinstance(v,float) else v for k,v in st.items() if k in ("prepare_seconds","interpret_seconds","gpu_seconds","host_seconds","early_seconds","early_rows","early_mapped","early_msgs","host_jobs_seconds","stage_seconds","total_seconds")})
PY
