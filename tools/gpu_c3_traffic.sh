# C3 roofline traffic: FETCH_SIZE and WRITE_SIZE passes (separate runs) over tools/c3_stage_pmc.py,
# plus a kernel trace of the same program.  -> gpurun_out/$1/{trace,pmc_fetch,pmc_write}
set -o pipefail
export TMPDIR=/tmp
T=${1:-r05_c3traffic}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd /tmp
P="python3 $GRAFT_REPO_ROOT/tools/c3_stage_pmc.py 10"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $P > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $P > $O/fetch.log 2>&1 || { tail $O/fetch.log; exit 2; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $P > $O/write.log 2>&1 || { tail $O/write.log; exit 3; }
cd $GRAFT_REPO_ROOT
python3 tools/summarize_prof.py $O > $O/summary.json || exit 4
python3 -c "
import json; d=json.load(open('$O/summary.json'))
for k,e in sorted(d['kernels'].items(), key=lambda x:-x[1].get('total_ns',0))[:14]:
    print(f\"{k:34s} calls {e.get('calls')} avg_us {e.get('avg_ns',0)/1e3:8.1f} fetch_launches {e.get('fetch_size_launches')} fetchx2/launch {e.get('fetch_bytes_x2_per_launch',0):.4g} write/launch {e.get('write_size_bytes_per_launch',0):.4g}\")
print(d.get('stages'))"
