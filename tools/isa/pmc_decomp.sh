#!/bin/bash
# PMC decomposition of the C2 ladder beside the isolated primitives (run via gpurun):
# three counter passes over one bench step and over tools/isa/prim_table.py, plus the
# single-asm-block microbenchmark ops.  usage: TAG
export TMPDIR=/tmp
T=${1:-r03c}
O=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/isa/ubench_table.py $O/ubench_asm.json 25,26,27,28,29,30,0,4 8,4,2,1 > $O/ubench_asm.log 2>&1 || { tail -20 $O/ubench_asm.log; exit 1; }
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
P2="SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS"
P3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES SQ_CYCLES SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/bench_p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-extra --sustain-s 0 --steps 1 --warmup 0 > /dev/null 2> $O/bench_p$i.err || { tail -5 $O/bench_p$i.err; exit 2; }
  timeout -s KILL 120 rocprofv3 --pmc $P -d $O/prim_p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/isa/prim_table.py $O/prim_p$i.json > /dev/null 2> $O/prim_p$i.err || { tail -5 $O/prim_p$i.err; exit 3; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-extra --sustain-s 0 --steps 3 --warmup 1 > $O/bench_trace.json 2> $O/trace.err || { tail -5 $O/trace.err; exit 4; }
cd $GRAFT_REPO_ROOT
python3 tools/isa/pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
