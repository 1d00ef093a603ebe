#!/bin/bash
# CPU-only build of tools/pipe_probe (the host engine + a sleeping device stub).
set -e
D=$(cd "$(dirname "$0")" && pwd)
R=$D/../..
mkdir -p $R/tools/_build
g++ -O3 -std=c++17 -march=native -pthread -I$R/include -I$R/rust-bitcoinconsensus_amd/csrc \
    -o $D/pipe_probe $D/pipe_probe.cpp $R/rust-bitcoinconsensus_amd/csrc/host/*.cpp
