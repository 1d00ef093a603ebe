#!/bin/bash
# Builds tools/host_prof (the host half of verify_batch with a stub device) and prints per-call wall
# and process CPU time at several host thread counts.  usage: tools/host_prof/run.sh OUT N THREADS...
OUT=$1; N=$2; shift 2
cd "$(dirname "$0")/../../rust-bitcoinconsensus_amd" || exit 1
S=$(ls csrc/host/*.cpp | grep -v taproot.cpp)
g++ -O3 -std=c++17 -w -I../include -Icsrc -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
    ../tools/host_prof/host_prof.cpp $S -o "$OUT" -lpthread || exit 1
for t in "$@"; do
  echo "== threads $t"
  BCC_HOST_THREADS=$t timeout -k 10 300 "$OUT" "$N" || exit 2
done
