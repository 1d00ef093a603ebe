"""Timeline of the ECDSA stage's kernels from a rocprofv3 kernel trace: for each stage run (a
batch_sinv launch starts one), every kernel's start and end in microseconds from the run's start.

    python3 tools/stage_timeline.py DIR_WITH_kernel_trace.csv_OR_results.db [GRID_MIN]

Only runs whose batch_sinv grid is at least GRID_MIN threads (default 32768: the 1M stage) are
shown; the last three are printed."""
import csv
import glob
import sqlite3
import sys


def main(d, grid_min):
    rows = []
    short = lambda nm: nm.split("(")[0].replace("bcc::", "").replace("(anonymous namespace)::", "")  # noqa: E731
    for p in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), grid))
    for p in glob.glob(f"{d}/**/*results.db", recursive=True):  # rocprofv3's default rocpd output
        for s, e, nm, gx in sqlite3.connect(p).execute("select start, end, name, grid_x from kernels"):
            rows.append((int(s), int(e), short(nm), int(gx)))
    if not rows:
        sys.exit(f"no kernel trace under {d}")
    rows.sort()
    runs, cur = [], None
    for s, e, name, grid in rows:
        if "batch_sinv" in name:
            cur = [] if grid >= grid_min else None
            if cur is not None:
                runs.append(cur)
        if cur is not None and ("ladder" in name or "keyq" in name or "fin" in name or "sinv" in name):
            cur.append((s, e, name, grid))
    for run in runs[-3:]:
        t0 = run[0][0]
        end = max(e for _, e, _, _ in run)
        print(f"run: {(end - t0) / 1e3:.1f} us")
        for s, e, name, grid in run:
            print(f"  {name[:34]:34s} grid {grid:9d}  {(s - t0) / 1e3:8.1f} -> {(e - t0) / 1e3:8.1f}  ({(e - s) / 1e3:7.1f})")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 32768)
