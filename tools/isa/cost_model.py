"""Issue-cost model of the signature kernels from a tools/isa/pmc_decomp.sh run:

    python3 tools/isa/cost_model.py gpurun_out/r03c > profiles/r03/ladder_cost_model.json

Per kernel and launch: VALU instructions by class from the PMC passes (SQ_INSTS_VALU_INT64 = the
v_mad_u64_u32 products, SQ_INSTS_VALU_INT32 = 32-bit integer ops: add-with-carry chains, shifts,
selects, ..., the rest = moves and other VALU), the GPU-busy cycles (GRBM_GUI_ACTIVE / 8 XCDs) and
the measured sustained issue cost of each class (tools/isa/ubench_table.py, 8 waves per SIMD,
8 independent instructions in one asm block: v_mad_u64_u32 / v_addc_co_u32 chains, v_add_u32 /
v_mov_b32).  predicted SIMD cycles = sum(count x cost) / SIMDs; compared with the measured cycles.
"""
import collections
import csv
import glob
import json
import os
import sys


def pmc(O):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(O, "*_p*", "**", "*counter_collection.csv"), recursive=True):
        src = "bench" if "/bench_p" in f else "prim"
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "").split("(")[0].replace("void ", "").replace("bcc::", "")
            agg[(src, k)][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(src, k, r["Counter_Name"])].add(r.get("Dispatch_Id", ""))
    out = {}
    for key, cs in agg.items():
        out[key] = {c: v / max(1, len(disp[(key[0], key[1], c)])) for c, v in cs.items()}
    return out


def main():
    O = sys.argv[1]
    ub = json.load(open(os.path.join(O, "ubench_asm.json")))
    simds = ub["cus"] * 4

    def cost(op, w=8):
        r = next(x for x in ub["rows"] if x["op"] == op and x["waves_per_simd"] == w)
        return r["cycles_per_wave_instr"], r
    c_mad, r_mad = cost(25)
    c_i32, _ = cost(29)
    c_oth, _ = cost(28)
    P = pmc(O)
    kernels = {}
    for (src, k), c in sorted(P.items()):
        if "SQ_INSTS_VALU" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        i64, i32 = c.get("SQ_INSTS_VALU_INT64", 0), c.get("SQ_INSTS_VALU_INT32", 0)
        oth = c["SQ_INSTS_VALU"] - i64 - i32
        pred = (i64 * c_mad + i32 * c_i32 + oth * c_oth) / simds
        meas = c["GRBM_GUI_ACTIVE"] / 8
        waves = c.get("SQ_WAVES", 0)
        kernels[f"{src}:{k}"] = dict(
            valu_per_wave=dict(int64_mad=i64 / waves if waves else None,
                               int32=i32 / waves if waves else None,
                               other=oth / waves if waves else None),
            valu_total=c["SQ_INSTS_VALU"], int64=i64, int32=i32, other=oth,
            salu=c.get("SQ_INSTS_SALU"), vmem_rd=c.get("SQ_INSTS_VMEM_RD"),
            salu_per_wave=c.get("SQ_INSTS_SALU", 0) / waves if waves else None,
            predicted_simd_cycles=pred, measured_simd_cycles=meas, predicted_over_measured=pred / meas,
            cycle_share=dict(int64_mad=i64 * c_mad / simds / pred, int32=i32 * c_i32 / simds / pred,
                             other=oth * c_oth / simds / pred),
            wait_any_over_wave_cycles=c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"] if c.get("SQ_WAVE_CYCLES") else None)
    out = dict(source=O, simds=simds,
               issue_cost_cycles_per_wave_instr=dict(int64_mad=c_mad, int32_carry=c_i32, other_full_rate=c_oth),
               mad_peak_measured=dict(rate_T=r_mad["rate_T"], clock_GHz=r_mad["clock_GHz"],
                                      at_2_4GHz_T=r_mad["rate_T"] * 2.4 / r_mad["clock_GHz"]),
               mad_peak_spec_T=2.4e9 * simds * 16 / 1e12, kernels=kernels)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
