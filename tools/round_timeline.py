"""Timeline of device rounds in a rocprofv3 kernel trace (one verify_batch call = one round).

    python3 tools/round_timeline.py DIR_WITH_kernel_trace.csv [--rounds 2] [--min-kernels 4]

Kernels are grouped into rounds wherever the device is idle for more than --gap-us (the host pass
between calls); the last --rounds rounds with at least --min-kernels kernels are printed with
start -> end times relative to the round's first kernel, and the median round span is reported."""
import argparse
import csv
import glob
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--min-kernels", type=int, default=4)
    ap.add_argument("--gap-us", type=float, default=300.0)
    ap.add_argument("--with", dest="with_", default=None,
                    help="keep only rounds containing a kernel whose name has this substring")
    a = ap.parse_args()
    ks = []
    for p in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        for row in csv.DictReader(open(p)):
            name = row["Kernel_Name"].split("(")[0]
            if "ubench" in name:
                continue
            ks.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), name,
                       row.get("Queue_Id", "?")))
    ks.sort()
    rounds, cur, end = [], [], None
    for k in ks:
        if cur and k[0] - end > a.gap_us * 1e3:
            rounds.append(cur)
            cur = []
        cur.append(k)
        end = k[1] if end is None or not cur[:-1] else max(end, k[1])
    if cur:
        rounds.append(cur)
    rounds = [r for r in rounds if len(r) >= a.min_kernels]
    if a.with_:
        rounds = [r for r in rounds if any(a.with_ in k[2] for k in r)]
    spans = [(max(k[1] for k in r) - r[0][0]) / 1e6 for r in rounds]
    print(f"{len(rounds)} rounds, span median {statistics.median(spans):.3f} ms, "
          f"min {min(spans):.3f} ms")
    for r in rounds[-a.rounds:]:
        t0 = r[0][0]
        print(f"-- round span {(max(k[1] for k in r) - t0) / 1e6:.3f} ms")
        for s, e, name, q in r:
            print(f"  {name[:40]:40s} queue {q:>3s} {(s - t0) / 1e6:7.3f} -> {(e - t0) / 1e6:7.3f}"
                  f"  ({(e - s) / 1e6:.3f})")


if __name__ == "__main__":
    main()
