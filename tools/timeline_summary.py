"""The last call of a rocprofv3 kernel + memory-copy trace as a text timeline (ms from the first
event of the window): python3 tools/timeline_summary.py TRACE_DIR WINDOW_MS"""
import csv
import glob
import os
import sys

d, win = sys.argv[1], float(sys.argv[2])
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for k in csv.DictReader(open(f)):
        ev.append((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K", k["Stream_Id"],
                   k["Kernel_Name"].split("(")[0].replace("bcc::(anonymous namespace)::", "").replace("bcc::", "")))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for m in csv.DictReader(open(f)):
        ev.append((int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "C", m.get("Stream_Id", ""),
                   m["Direction"] + " " + str(round(int(m.get("Bytes", m.get("Size", 0)) or 0) / 1e6, 2)) + " MB"))
ev.sort()
end = max(e[1] for e in ev)
sel = [e for e in ev if e[1] >= end - win * 1e6]
b = sel[0][0]
busy = 0
last_end = b
for s, e, t, st, n in sel:
    if t == "K":
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    print(f"{(s - b) / 1e6:8.3f} {(e - b) / 1e6:8.3f} {(e - s) / 1e6:7.3f} {t} {st:>3} {n}")
print(f"# window {(end - b) / 1e6:.2f} ms, kernels busy (union) {busy / 1e6:.2f} ms")
