set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_block_gpu.py tests/test_consensus_gpu.py tests/test_workload_gpu.py > gpurun_out/r05d/pytest.log 2>&1 || { grep -v "^  File" gpurun_out/r05d/pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/r05d/pytest.log
O=gpurun_out/r05d/ab
mkdir -p $O
for i in 1 2 3; do for e in 0 1; do
  BCC_EARLY_Q=$e timeout -k 10 200 python3 bench.py --config c3 --no-cpu --steps 300 --warmup 30 > $O/c3_e${e}_$i.json 2> $O/c3_e${e}_$i.err || { tail -5 $O/c3_e${e}_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_e${e}_$i.json')); b=d['batch_stats']; print('early=$e', $i, round(d['value']/1e6,3), round(d['ms_per_step'],3), 'host', round(b['host_seconds']*1e3,3), 'gpu', round(b['gpu_seconds']*1e3,3), 'interp', round(b['interpret_seconds']*1e3,3), 'early', b.get('early_rows'), b.get('early_mapped'), round(b.get('early_seconds',0)*1e3,3))"
done; done
bash tools/c3_copy_trace.sh r05d/copy && python3 tools/copy_timeline.py gpurun_out/r05d/copy/trace > gpurun_out/r05d/copy_timeline.txt 2>&1; head -24 gpurun_out/r05d/copy_timeline.txt
