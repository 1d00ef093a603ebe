"""Per-kernel durations of the full-size launches in a rocprofv3 kernel trace.

    python3 tools/trace_step.py DIR_WITH_kernel_trace.csv

bench.py also runs small launches (single calls, the drop-in's rounds), which skew the averages
of `--stats`; this keeps, per kernel, only the launches with that kernel's largest grid and
reports their count and median / min duration in microseconds, sorted by total time."""
import csv
import glob
import statistics
import sys


def main(d):
    paths = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not paths:
        sys.exit(f"no kernel_trace.csv under {d}")
    per = {}
    for p in paths:
        for row in csv.DictReader(open(p)):
            name = row["Kernel_Name"]
            if "ubench" in name or "rocclr" in name:
                continue
            grid = tuple(int(row[k]) for k in row if k.startswith("Grid_Size"))
            dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            per.setdefault(name.split("(")[0], []).append((grid, dur))
    rows = []
    for name, v in per.items():
        g = max(x[0] for x in v)
        ds = [x[1] for x in v if x[0] == g]
        rows.append((statistics.median(ds) * len(ds), name, len(ds), statistics.median(ds), min(ds), g))
    for _, name, n, med, mn, g in sorted(rows, reverse=True):
        print(f"{name[:60]:60s} n {n:4d} median_us {med:9.1f} min_us {mn:9.1f} grid {g}")


if __name__ == "__main__":
    main(sys.argv[1])
