# Drop-in leg: the bench process vs the standalone tool on one box (round 6 diagnosis).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06c}; mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $O/thp.txt 2>&1
cat $O/thp.txt
for rep in 1 2; do
  timeout -k 10 200 env PHASES=1 python3 tools/dropin_e2e.py 1000000 20 >> $O/dropin.txt 2>&1 || { tail -5 $O/dropin.txt; exit 1; }
  timeout -k 10 300 python3 bench.py --no-cpu --no-side --steps 5 --warmup 2 --sustain-s 0 > $O/bench_noside_$rep.json 2> $O/bench_noside_$rep.err || { tail -5 $O/bench_noside_$rep.err; exit 2; }
  timeout -k 10 300 python3 bench.py --no-cpu --steps 5 --warmup 2 --sustain-s 0 > $O/bench_side_$rep.json 2> $O/bench_side_$rep.err || { tail -5 $O/bench_side_$rep.err; exit 3; }
  grep -v amdgpu.ids $O/dropin.txt | tail -3
  python3 tools/bench_summary.py $O/bench_noside_$rep.json $O/bench_side_$rep.json | grep -v c3_ | grep -v c4_
done
