#!/bin/bash
# A/B of engine library variants on the GPU box (run via gpurun).  Each variant is a full build of
# librbc_amd.so under variants/NAME/ (git-ignored; it travels with the snapshot), e.g.
#   make -C rust-bitcoinconsensus_amd BUILD=../variants/v5_640/obj \
#        OPT="-O3 -DBCC_LADDER_WAVES=5 -DBCC_LADDER_WG=640" && mv .../librbc_amd.so variants/v5_640/
#   gpurun -- 'bash tools/varrun.sh base v5_640'   -> gpurun_out/var/NAME_CONFIG.json
# The box's copy of the tree is scratch, so swapping the in-tree library there is harmless.
mkdir -p gpurun_out/var
for v in "${@:-base}"; do
  cp variants/$v/librbc_amd.so rust-bitcoinconsensus_amd/librbc_amd.so || exit 1
  for c in c2 c5; do
    timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/var/${v}_$c.json 2> gpurun_out/var/${v}_$c.err || exit 1
  done
done
