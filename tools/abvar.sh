#!/bin/bash
# Build an engine-library variant for A/B runs:  tools/abvar.sh NAME "EXTRA HIPCC FLAGS"
#   -> abvar/NAME/librbc_amd.so  (git-ignored; travels with the gpurun snapshot)
# Run on the GPU box:  bash tools/ab_run.sh ROUNDS NAME1 NAME2 ...  -> gpurun_out/ab/NAME_i.json
set -e
NAME=$1
FLAGS=${2:-}
mkdir -p abvar/$NAME
make -s -C rust-bitcoinconsensus_amd BUILD=../abvar/$NAME/obj OPT="-O3 $FLAGS" librbc_amd.so -j8
mv rust-bitcoinconsensus_amd/librbc_amd.so abvar/$NAME/librbc_amd.so
# restore the in-tree product build
make -s -C rust-bitcoinconsensus_amd -j8
