set -o pipefail
for rep in 1 2; do for r in 131072 81920 65536 49152; do
BCC_TAPROOT_ROUND=$r timeout -k 10 120 python3 tools/e2e_timeline.py c5t 10 2>&1 | grep -E "ms per call" | sed "s/^/round $r: /"
done; done
