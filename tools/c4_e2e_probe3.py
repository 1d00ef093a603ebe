"""bench.py's C4 drop-in leg: torch.cuda.set_stream (as bench.py does) vs not (probe)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import bitcoinconsensus_amd as B  # noqa: E402

torch.cuda.set_device(0)
B.set_device(0)
job = bench.TupleJob(B, bench.DEFAULT_N["c4"], bench.SEEDS["c4"], 0, "c4", first=0, total=bench.DEFAULT_N["c4"])
h = job.ts.host()
print("fresh:", job.end_to_end(h)["calls_ms"], flush=True)
n_valid = job.valid()
print("after valid():", job.end_to_end(job.ts.host())["calls_ms"], flush=True)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
print("after torch.cuda.set_stream:", job.end_to_end(job.ts.host())["calls_ms"], flush=True)
