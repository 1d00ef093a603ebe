"""Per-kernel sums of the PMC passes written by tools/isa/pmc_decomp.sh (one line per kernel of
interest: the C2 ladder and the primitive kernels), per launch."""
import collections
import csv
import glob
import os
import sys

O = sys.argv[1]
KEEP = ("twist_ladder", "twist_keyq", "prim_kernel", "ecdsa_tprep", "batch_sinv", "twist_fin",
        "bip143")


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in sorted(glob.glob(os.path.join(O, "*_p*", "**", "*counter_collection.csv"), recursive=True)):
        src = "bench" if "/bench_p" in f else "prim"
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if not any(x in k for x in KEEP):
                continue
            short = k.split("(")[0].replace("void ", "").replace("bcc::", "")
            key = (src, short)
            agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
            launches[(key, r["Counter_Name"])].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    for key in sorted(agg):
        per = {}
        for c, v in agg[key].items():
            n = max(1, len(launches[(key, c)]))
            per[c] = v / n
        n = max(len(launches[(key, c)]) for c in agg[key])
        print(f"{key[0]:5s} {key[1]:40s} launches~{n}")
        for c in sorted(per):
            print(f"      {c:26s} {per[c]:.5g}")


if __name__ == "__main__":
    main()
