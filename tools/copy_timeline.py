"""Per-call timeline of a C3 run from a rocprofv3 --kernel-trace --memory-copy-trace directory:
copies (direction, bytes unknown: duration only) and kernels merged in time order, for the last
`--calls` verify_batch rounds (a round starts at an H2D copy that follows a D2H copy).

    python3 tools/copy_timeline.py gpurun_out/TAG/trace [--calls 2]
"""
import csv
import os
import sys


def load(d):
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"].split("(")[0][:44],
                   r.get("Stream_Id", "")))
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "C " + r["Direction"].replace("MEMORY_COPY_", ""), r.get("Stream_Id", "")))
    ev.sort()
    return ev


def main():
    d = sys.argv[1]
    calls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 2
    ev = load(d)
    # round boundaries: a DEVICE_TO_HOST copy closes a round
    ends = [i for i, e in enumerate(ev) if "DEVICE_TO_HOST" in e[2]]
    if len(ends) < calls + 1:
        print("not enough rounds")
        return
    for c in range(calls, 0, -1):
        a, b = ends[-c - 1] + 1, ends[-c] + 1
        t0 = ev[a][0]
        print(f"-- round: {(ev[b - 1][1] - t0) / 1e3:.1f} us from first event to the verdict copy; "
              f"gap before it {(t0 - ev[a - 1][1]) / 1e3:.1f} us")
        for s, e, n, st in ev[a:b]:
            print(f"  {n:52s} s{st:>2} {(s - t0) / 1e3:9.1f} -> {(e - t0) / 1e3:9.1f}  ({(e - s) / 1e3:7.1f} us)")


if __name__ == "__main__":
    main()
