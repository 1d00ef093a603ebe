set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/qp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/qp/pytest.log 2>&1 || { tail -30 gpurun_out/qp/pytest.log; exit 1; }
tail -2 gpurun_out/qp/pytest.log
timeout -k 10 300 python3 tools/keyq_sweep.py 10 > gpurun_out/qp/sweep_qp1.txt 2>&1 || exit 2
cat gpurun_out/qp/sweep_qp1.txt
BENCH_ARGS="--steps 20 --warmup 10 --no-cpu --no-extra" bash tools/ab_run.sh 3 c2 qp0 qp1 2>&1 | tee gpurun_out/qp/ab_c2.txt
