set -o pipefail
run() { timeout -k 10 200 env "$@" python3 bench.py --config c3 --no-cpu --no-extra --steps 300 --warmup 30 2>/dev/null | python3 -c "import json,sys; print('$*', round(json.load(sys.stdin)['value']/1e6,3))"; }
for rep in 1 2 3 4; do run BCC_EARLY_SIGHASH=0 || exit 1; run BCC_EARLY_SIGHASH_MIN=64 || exit 1; run BCC_EARLY_SIGHASH_MIN=96 || exit 1; done
