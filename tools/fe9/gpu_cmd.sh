export TMPDIR=/tmp
timeout -k 10 200 python tools/fe9/run.py 2 3 > gpurun_out/fe9_r2.txt 2>&1 || exit 1
timeout -k 10 100 python tools/fe9/run_ub2.py > gpurun_out/ub2b.txt 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/fe9pmc -o run --output-format csv -- python tools/fe9/run.py 2 > /dev/null 2> gpurun_out/fe9pmc.err || exit 3
cat gpurun_out/fe9_r2.txt gpurun_out/ub2b.txt
