set -o pipefail
for r in 131072 65536 262144; do
BCC_TAPROOT_TRACE=1 BCC_TAPROOT_ROUND=$r timeout -k 10 120 python3 tools/e2e_timeline.py c5t 6 2>&1 | grep -E "taproot rounds|ms per call" | tail -3
done
