#!/bin/bash
# Round 3, GPU pass J: -m gpu suite; the fused sighash front + split ladder A/B on C3 and C2
# (BCC_LADDER_SPLIT); a C3 kernel trace (timeline of one verify_batch round).
export TMPDIR=/tmp
O=gpurun_out/${1:-r03j}
T=$(basename $O)
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/ab_env.sh $T 3 c3 - BCC_LADDER_SPLIT=0 || exit 2
bash tools/ab_env.sh $T 2 c2 - BCC_LADDER_SPLIT=0 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c3trace -o run --output-format csv -- python bench.py --config c3 --steps 3 --warmup 1 --no-cpu > $O/c3_under_trace.json 2> $O/c3trace.err || { tail -5 $O/c3trace.err; exit 4; }
echo done
