#!/bin/bash
# Build both libraries of a variant for primitive + bench A/Bs:  tools/abvar_both.sh NAME "FLAGS"
#   -> abvar/NAME/{librbc_amd.so,librbc_bench.so} (git-ignored; they travel with the gpurun snapshot)
# On the box, tools/ab_prim.sh ROUNDS NAME... swaps them into the package directory in turn.
set -e
NAME=$1
FLAGS=${2:-}
mkdir -p abvar/$NAME
make -s -C rust-bitcoinconsensus_amd BUILD=../abvar/$NAME/obj OPT="-O3 $FLAGS" librbc_amd.so librbc_bench.so -j8
mv rust-bitcoinconsensus_amd/librbc_amd.so rust-bitcoinconsensus_amd/librbc_bench.so abvar/$NAME/
# restore the in-tree product build
make -s -C rust-bitcoinconsensus_amd -j8
