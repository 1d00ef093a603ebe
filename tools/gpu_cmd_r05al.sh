set -o pipefail
BCC_TUPLE_TRACE=1 timeout -k 10 400 python bench.py --config c4 --no-cpu > gpurun_out/r05al_c4.json 2> gpurun_out/r05al_c4.err || { tail -20 gpurun_out/r05al_c4.err; exit 1; }
grep "tuple_rounds:" gpurun_out/r05al_c4.err | tail -3
BCC_TUPLE_TRACE=1 timeout -k 10 300 python3 tools/c4_e2e_probe.py 2>&1 | grep "tuple_rounds:\|calls\|runs" | tail -5
