#!/bin/bash
# Round 3, GPU pass A: sighash goldens on the GPU, the counter list, the sustained microbenchmark
# table and a clock/issue PMC pass over the C2 ladder.  usage: TAG
export TMPDIR=/tmp
T=${1:-r03a}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sighash_goldens.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_sighash.log 2>&1 || { tail -30 $O/pytest_sighash.log; exit 1; }
tail -2 $O/pytest_sighash.log
timeout -k 10 120 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 300 python -u tools/isa/ubench_table.py $O/ubench_sustained.json > $O/ubench.log 2>&1 || { tail -20 $O/ubench.log; exit 2; }
cat $O/ubench.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(f\"{d['name']:36s} w{d['waves_per_simd']} {d['rate_T']:7.2f} T/s clk {d['clock_GHz']:.3f} cyc {d['cycles_per_wave_instr']:.2f}\")"
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 1 --warmup 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/$O/pmc_sq -o run --output-format csv -- $B > /dev/null 2> $GRAFT_REPO_ROOT/$O/pmc_sq.err || { tail -5 $GRAFT_REPO_ROOT/$O/pmc_sq.err; exit 3; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o run --output-format csv -- $B > /dev/null 2> $GRAFT_REPO_ROOT/$O/trace.err || { tail -5 $GRAFT_REPO_ROOT/$O/trace.err; exit 4; }
echo done
