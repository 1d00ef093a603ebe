"""Sustained per-instruction issue costs on this GPU (run on the GPU box):

    python3 tools/isa/ubench_table.py OUT.json [OPS,..] [WAVES,..]

For every microbenchmark op (csrc/bench/microbench.hip) at 8 and 4 waves per SIMD: launches of
~20 ms back to back for >= 1 s, then the median of 3 timed launches; reports lane-instructions/s,
the in-kernel clock (s_memtime / s_memrealtime) and the cost in SIMD cycles per wave-instruction
= clock x SIMDs x 64 / rate (2 = full rate for wave64, 4 = half rate)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rust-bitcoinconsensus_amd")]
import bitcoinconsensus_amd as B  # noqa: E402

OPS = {0: "v_mad_u64_u32", 1: "v_mul_lo_u32", 2: "v_mul_hi_u32", 3: "v_add_co_u32 (sgpr)",
       4: "v_addc_co_u32", 5: "v_mad_u32_u24", 6: "v_lshl_add_u64", 8: "v_add_u32",
       9: "v_add3_u32", 10: "v_mul_u32_u24", 12: "v_alignbit_b32", 13: "v_lshrrev_b64",
       14: "v_add_co_u32 (vcc)", 15: "v_cndmask_b32 (vcc)", 16: "mad_u64_u32+addc pair",
       18: "mad_u64_u32+add_u32 pair", 19: "v_mov_b32", 20: "addc chain (1 dependent chain)",
       21: "mad+addc chain (1 dependent chain)", 22: "v_cndmask_b32_e64 (sgpr mask)",
       23: "v_subb_co_u32", 24: "mad+s_nop 1+addc",
       25: "8 mad_u64, own SGPR carries, 1 asm", 26: "8 addc_e64 chains, own SGPR carries, 1 asm",
       27: "4 (mad->vcc->addc) pairs, 1 asm", 28: "8 v_add_u32, 1 asm",
       29: "8 addc_e32, one VCC chain, 1 asm", 30: "8 mad_u64 carry->vcc, 1 asm"}


def main():
    import torch
    torch.cuda.init()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    simds = cus * 4
    out = dict(cus=cus, rows=[])
    first = True
    ops = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else list(OPS)
    waves = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [8, 4]
    for op in ops:
        name = OPS[op]
        for w in waves:
            rate, clk, ms = B.microbench_sustained(op, w, 20.0, 2.0 if first else 1.0, 3)
            first = False
            cyc = clk * 1e9 * simds * 64 / rate
            row = dict(op=op, name=name, waves_per_simd=w, rate_T=round(rate / 1e12, 3),
                       clock_GHz=round(clk, 3), launch_ms=round(ms, 2),
                       cycles_per_wave_instr=round(cyc, 3))
            out["rows"].append(row)
            print(json.dumps(row), flush=True)
    json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
