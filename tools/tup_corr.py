"""Host events (BCC_TUPLE_TRACE 'tup' lines) merged with the rocprofv3 kernel / copy trace of the
last bcc_pubkey_verify_batch call: python3 tools/tup_corr.py OUT_DIR (run.log + tl/)."""
import csv
import glob
import re
import sys

d = sys.argv[1]
ev = []
for f in glob.glob(d + '/tl/**/*kernel_trace.csv', recursive=True):
    for k in csv.DictReader(open(f)):
        ev.append((int(k['Start_Timestamp']), int(k['End_Timestamp']), 'K' + k['Stream_Id'], k['Kernel_Name'].split('(')[0].split('::')[-1]))
for f in glob.glob(d + '/tl/**/*memory_copy_trace.csv', recursive=True):
    for m in csv.DictReader(open(f)):
        ev.append((int(m['Start_Timestamp']), int(m['End_Timestamp']), 'C' + m.get('Stream_Id', ''), m['Direction'][12:]))
host = []
for line in open(d + '/run.log'):
    m = re.match(r'\[bcc\] tup k=(\d+) (.*) (\d+)$', line.strip())
    if m:
        host.append((int(m.group(3)), int(m.group(3)), 'H', f"k={m.group(1)} {m.group(2)}"))
starts = [e[0] for e in host if e[3].startswith('k=0 m=')]
b = starts[-1] - 3_000_000
for s, e, t, n in sorted(ev + host):
    if b <= s < b + 100e6:
        print(f"{(s - b) / 1e6:8.3f} {(e - b) / 1e6:8.3f} {(e - s) / 1e6:7.3f} {t:3} {n}")
