"""The last drop-in call's device rounds from a rocprofv3 --kernel-trace --memory-copy-trace run
(rocpd results.db): kernels and copy bursts on one time axis, microseconds from the window start.
    python3 tools/dropin_timeline.py RESULTS_DB [WINDOW_MS]"""
import sqlite3
import sys


def main(db, window_ms):
    c = sqlite3.connect(db)
    ev = [(s, e, "COPY", sz) for s, e, sz in c.execute("select start, end, size from memory_copies")]
    ev += [(s, e, n.split("(")[0].replace("bcc::", ""), g)
           for s, e, n, g in c.execute("select start, end, name, grid_x from kernels")]
    ev.sort()
    end = max(e for _, e, _, _ in ev)
    last = [x for x in ev if x[0] > end - window_ms * 1e6]
    t0 = last[0][0]
    bursts, cur = [], None
    for s, e, n, sz in last:
        if n != "COPY":
            continue
        if cur and s - cur[1] < 200e3:
            cur = [cur[0], max(cur[1], e), cur[2] + 1, cur[3] + sz]
        else:
            if cur:
                bursts.append(cur)
            cur = [s, e, 1, sz]
    if cur:
        bursts.append(cur)
    rows = [(b[0], b[1], f"copies x{b[2]} {b[3] / 1e6:.1f} MB ({b[3] / max(1, b[1] - b[0]):.1f} GB/s)", "")
            for b in bursts]
    rows += [x for x in last if x[2] != "COPY"]
    for s, e, n, g in sorted(rows):
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n[:48]:48s} {g}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 25)
