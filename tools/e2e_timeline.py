"""One bench config's timed step, called back to back (no profiler-visible extras), for a
rocprofv3 --kernel-trace --memory-copy-trace timeline:  python3 tools/e2e_timeline.py c5t|c3|c2 CALLS
Prints the wall time of every call."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bench  # noqa: E402
import bitcoinconsensus_amd as B  # noqa: E402

cfg = sys.argv[1]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
cls = {"c2": bench.C2, "c3": bench.C3, "c5t": bench.C5T}[cfg]
job = cls(B, bench.DEFAULT_N[cfg], bench.SEEDS[cfg], 0)
if cfg == "c2":
    job.step = lambda sp: job.wl.verify_batch()  # the drop-in leg
ts = []
for _ in range(calls):
    t0 = time.perf_counter()
    job.step(None)
    ts.append((time.perf_counter() - t0) * 1e3)
print(cfg, "ms per call:", [round(t, 2) for t in ts], flush=True)
