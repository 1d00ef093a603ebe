set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_field_gpu.py > gpurun_out/field_v4.log 2>&1 || { tail -30 gpurun_out/field_v4.log; exit 1; }
tail -3 gpurun_out/field_v4.log
bash tools/ab_prim.sh 2 c2 base v4 2>&1 | tee gpurun_out/ab_v4.txt
