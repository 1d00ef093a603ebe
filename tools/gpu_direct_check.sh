# The direct upload after its per-array size rule: GPU suite, C3 (BCC_DIRECT_UPLOAD 0 / 1 in
# alternating processes), the C2 drop-in alternating call by call in one process.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-dcheck}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_bench_ab.sh ${1:-dcheck}_c3 3 "--config c3 --no-cpu --steps 20 --warmup 5 --sustain-s 0" BCC_DIRECT_UPLOAD=0 BCC_DIRECT_UPLOAD=1 || exit 2
timeout -k 10 300 python3 tools/dropin_interleave.py 1000000 12 500000:0:1:1:0 500000:0:1:1:1 > $O/interleave.txt 2>&1 || { tail -20 $O/interleave.txt; exit 3; }
cat $O/interleave.txt
