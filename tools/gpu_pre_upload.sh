# Per-shard row pre-upload (bcc_set_pre_upload): GPU suite, a copy/kernel trace of the drop-in, and
# the switch alternating call by call in one process (two processes), then one C2 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-preup}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run -- python3 tools/dropin_e2e.py 1000000 4 > $O/trace.txt 2>&1 || exit 2
python3 tools/dropin_timeline.py $O/trace/run_results.db 12 > $O/timeline.txt
bash tools/gpu_dropin_settings.sh ${1:-preup}_ab 2 500000:0:1:1:1:0:0 500000:0:1:1:1:0:1
