set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
for rep in 1 2; do
  for t in "" 1 stream; do
    timeout -k 10 200 env PHASES=1 DROPIN_TORCH=$t python3 tools/dropin_e2e.py 1000000 20 >> $O/dropin.txt 2>&1 || { tail -5 $O/dropin.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/dropin.txt
