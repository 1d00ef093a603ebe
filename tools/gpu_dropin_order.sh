# Drop-in leg of the C2 line vs what ran before it in the process (round 6 diagnosis).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r06d}; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 300 env "$@" python3 bench.py --no-cpu --steps 5 --warmup 2 --sustain-s 0 $EXTRA > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -5 $O/bench_$tag.err; exit 2; }; python3 tools/bench_summary.py $O/bench_$tag.json | grep -v "c3_\|c4_\|placement"; }
for rep in 1 2; do
  EXTRA="--no-side" run noside_$rep X=1
  EXTRA="--side-c4 0" run c3only_$rep X=1
  EXTRA="" run side_$rep X=1
  EXTRA="" run side_early_$rep BCC_BENCH_DROPIN_EARLY=1
done
