#!/bin/bash
# Kernel trace + SQ / FETCH_SIZE / WRITE_SIZE passes (tools/profile_c2.sh, FULL=1) of the C2, C4 and
# C5 bench steps on the current tree (run via gpurun).  usage: tools/profile_final.sh TAG
T=${1:-r04z}
export FULL=1
bash tools/profile_c2.sh ${T}_c2 || exit 1
bash tools/profile_c2.sh ${T}_c4 --config c4 || exit 2
bash tools/profile_c2.sh ${T}_c5 --config c5 || exit 3
