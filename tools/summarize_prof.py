"""Summarise a tools/profile_round.sh output directory: per-kernel launches / average duration
from the --kernel-trace --stats pass and per-launch FETCH_SIZE / WRITE_SIZE from the --pmc passes
(rocprofv3 reports both in KB; gfx950 FETCH_SIZE counts 128-B requests as 64 B for wide
coalesced reads, MI355X_MICROARCH.md "HBM", so `fetch_bytes_x2` doubles it)."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("bcc::", "").replace("(anonymous namespace)::", "")


def main(d):
    out = {"kernels": {}}
    stats = glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True)
    for f in stats:
        for r in csv.DictReader(open(f)):
            out["kernels"].setdefault(short(r["Name"]), {}).update(
                calls=int(r["Calls"]), avg_ns=float(r["AverageNs"]), total_ns=float(r["TotalDurationNs"]))
    for tag, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        agg, cnt = collections.defaultdict(float), collections.Counter()
        for f in glob.glob(os.path.join(d, tag, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] != ctr:
                    continue
                k = short(r["Kernel_Name"])
                agg[k] += float(r["Counter_Value"])
                cnt[k] += 1
        for k in agg:
            e = out["kernels"].setdefault(k, {})
            e[ctr.lower() + "_bytes_per_launch"] = agg[k] * 1024 / cnt[k]
            e[ctr.lower() + "_launches"] = cnt[k]
            e[ctr.lower() + "_bytes_total"] = agg[k] * 1024
    # SQ / GRBM issue counters (pmc_sq pass): per launch, per kernel
    sq, sqn = collections.defaultdict(float), collections.Counter()
    for f in glob.glob(os.path.join(d, "pmc_sq", "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            sq[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            key = (k, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            if key not in seen:
                seen.add(key)
                sqn[k] += 1
    for (k, c), v in sq.items():
        e = out["kernels"].setdefault(k, {})
        e.setdefault("pmc_per_launch", {})[c] = v / max(1, sqn[k])
        e["pmc_launches"] = sqn[k]
    for k, e in out["kernels"].items():
        if "fetch_size_bytes_per_launch" in e:
            e["fetch_bytes_x2_per_launch"] = 2 * e["fetch_size_bytes_per_launch"]
    # per signature stage = all launches of one run_ecdsa / schnorr call.  The PMC passes run
    # bench.py --steps 1 --warmup 0: one timed step + 3 HIP-event timing repetitions = 4 stages,
    # plus, for the C2 line (which carries drop_in_end_to_end), 3 drop-in verify_batch runs over
    # the same inputs = 7.  A stage may launch a kernel once per lane chunk (C4 at 8M, C5 at 16M).
    stages = {"ecdsa": ["batch_sinv_kernel", "ecdsa_tprep_kernel", "twist_keyq_kernel", "twist_keyq2_kernel",
                        "twist_ladder_g_kernel", "void twist_ladder_kernel<false>",
                        "void twist_fin_kernel<false>"],
              "schnorr": ["schnorr_tladder_kernel", "schnorr_tprep_kernel", "void twist_ladder_kernel<true>",
                          "void twist_fin_kernel<true>"]}
    K = out["kernels"]
    bench = os.path.join(d, "bench_under_rocprof.json")
    if os.path.exists(bench):
        try:
            out["bench_under_rocprof"] = json.loads(open(bench).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            pass
    n_default = 7 if "drop_in_end_to_end" in out.get("bench_under_rocprof", {}) else 4
    for st, ks in stages.items():
        if not any("fetch_size_launches" in K.get(k, {}) for k in ks):
            continue
        # at least one launch of each stage kernel per execution (one lane chunk; round 6: K_keyq
        # and K_tladder_g twice when K_keyq is split at the last whole residency round): the
        # smallest launch count (K_inv / K_tfin) is the execution count
        nl = {K[k]["fetch_size_launches"] for k in ks if "fetch_size_launches" in K.get(k, {})}
        n_stage = min(nl) if nl else n_default
        fb = sum(K[k].get("fetch_size_bytes_total", 0) for k in ks if k in K) / n_stage
        wb = sum(K[k].get("write_size_bytes_total", 0) for k in ks if k in K) / n_stage
        out.setdefault("stages", {})[st] = dict(executions=n_stage, fetch_bytes=fb, fetch_bytes_x2=2 * fb,
                                               write_bytes=wb, traffic_bytes=2 * fb + wb)
        # per stage execution from the PMC launches (bench.py --no-extra runs: every stage full-size)
        fl = sum(K[k].get("fetch_size_bytes_total", 0) for k in ks if k in K) / n_stage
        wl = sum(K[k].get("write_size_bytes_total", 0) for k in ks if k in K) / n_stage
        out["stages"][st].update(per_launch_fetch_bytes_x2=2 * fl, per_launch_write_bytes=wl,
                                 per_launch_traffic_bytes=2 * fl + wl,
                                 kernels=[k for k in ks if k in K])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
