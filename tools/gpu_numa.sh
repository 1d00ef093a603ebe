#!/bin/bash
# Drop-in end to end vs CPU placement (run via gpurun): default affinity, then the CPUs of the
# GPU's NUMA node only, then the other node; one e2e_cgroup process per setting, interleaved.
export TMPDIR=/tmp
O=gpurun_out/${1:-r03n}
mkdir -p $O
nodes=$(ls -d /sys/devices/system/node/node* 2>/dev/null | wc -l)
gnode=$(cat /sys/class/drm/card*/device/numa_node 2>/dev/null | grep -v -- -1 | head -1)
echo "numa nodes $nodes, gpu node ${gnode:-?}" | tee $O/numa.txt
for n in $(ls -d /sys/devices/system/node/node* 2>/dev/null); do echo "$(basename $n): $(cat $n/cpulist)"; done | tee -a $O/numa.txt
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))" | tee -a $O/numa.txt
g=${gnode:-0}; other=$(( (g + 1) % (nodes > 0 ? nodes : 1) ))
gl=$(cat /sys/devices/system/node/node$g/cpulist 2>/dev/null)
ol=$(cat /sys/devices/system/node/node$other/cpulist 2>/dev/null)
for rep in 1 2; do
  for mode in default gpu_node other_node; do
    case $mode in
      default) pre="";;
      gpu_node) pre="taskset -c $gl";;
      other_node) pre="taskset -c $ol";;
    esac
    [ -n "$pre" ] && [ -z "$gl" ] && continue
    echo "== $mode rep $rep" >> $O/e2e.txt
    timeout -k 10 200 $pre python -u tools/e2e_cgroup.py 1000000 0:0 >> $O/e2e.txt 2>&1 || { tail -5 $O/e2e.txt; exit 1; }
    echo "$mode $rep $(grep best_ms $O/e2e.txt | tail -1)"
  done
done
