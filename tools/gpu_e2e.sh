#!/bin/bash
# Drop-in end to end on the GPU box (run via gpurun): verify_batch on the C2 inputs with the
# cgroup / rusage accounting of tools/e2e_cgroup.py for several (pipeline chunk : host threads)
# configurations, with and without the persistent host teams (BCC_HOST_TEAM), then the C3 block
# replay both ways.   usage: tools/gpu_e2e.sh TAG [chunk:threads ...]
export TMPDIR=/tmp
T=${1:-r03e}; shift
O=gpurun_out/$T
mkdir -p $O
CFG=${@:-0:0 262144:0 524288:0 262144:12 0:12}
timeout -k 10 300 python -u -m pytest tests/test_block_gpu.py tests/test_consensus_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_block.log 2>&1 || { tail -30 $O/pytest_block.log; exit 1; }
tail -1 $O/pytest_block.log
for team in 1 0; do
  BCC_HOST_TEAM=$team timeout -k 10 300 python -u tools/e2e_cgroup.py 1000000 $CFG > $O/e2e_team$team.txt 2>&1 || { tail -20 $O/e2e_team$team.txt; exit 2; }
  grep best_ms $O/e2e_team$team.txt | sed "s/^/team$team /"
done
# C3: persistent teams on / off, long chains on the host (default 32 blocks) / all on the GPU (0)
i=0
for v in "1 32" "0 32" "1 0" "1 32"; do
  set -- $v
  i=$((i+1)); tag=team$1_chain$2_$i
  BCC_HOST_TEAM=$1 BCC_HOST_CHAIN_BLOCKS=$2 timeout -k 10 300 python bench.py --config c3 --no-cpu > $O/bench_c3_$tag.json 2> $O/bench_c3_$tag.err || { tail -20 $O/bench_c3_$tag.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/bench_c3_$tag.json')); b=d.get('batch_stats',{}); print('c3 $tag', round(d['value']/1e6,3), round(d['ms_per_step'],3), {k: (round(v*1e3,3) if k.endswith('seconds') else v) for k,v in b.items()})"
done
