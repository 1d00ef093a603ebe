"""One-line summary of a bench.py JSON line (tools/gpu_run.sh)."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads([ln for ln in open(f) if ln.startswith("{")][-1])
    r = d["roofline"]
    cb = d.get("cpu_baseline") or {}
    print(f.split("/")[-1], d["config"]["workload"][:3], round(d["value"] / 1e6, 3), d["unit"],
          "ms", round(d["ms_per_step"], 3), "frac", round(r["frac"], 4),
          "stage_ms", round(r.get("per_launch", {}).get("avg_ms", 0), 3),
          "cpu", round(cb.get("value", 0)), "mism", cb.get("gpu_verdict_mismatches"))
    e = d.get("drop_in_end_to_end")
    if e and "inputs_per_s" in e:
        print("  drop-in", round(e["inputs_per_s"] / 1e6, 2), "sustained",
              round(e["sustained_inputs_per_s"] / 1e6, 2), "cpu_s/M",
              round(e["sustained_cpu_s_per_M"], 3), "busy", round(e.get("sustained_cpus_busy", 0), 1))
        if e.get("phases"):
            print("  phases", {k: v for k, v in e["phases"].items() if k != "note"})
        if e.get("host_placement"):
            print("  placement", e["host_placement"], "machine", e.get("machine"))
    for k in ("c3_block_replay", "c4_pubkey_verify_batch"):
        x = d.get(k)
        if x:
            rate = x.get("inputs_per_s") or x.get("verifies_per_s")
            print(" ", k, round(rate / 1e6, 3), "M/s", "ms", round(x.get("ms_median") or x.get("ms"), 2),
                  "x cpu", round(x.get("gpu_vs_cpu", 0), 1),
                  "mism", x.get("gpu_verdict_mismatches_all_items", x.get("mismatches_vs_staged")))
