"""bench.py's C4 drop-in leg after bench's own sequence (torch stream, timed staged steps, HIP-event
kernel times, microbench): which step slows bcc_pubkey_verify_batch's GPU waits (probe)."""
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
job = bench.TupleJob(B, bench.DEFAULT_N["c4"], bench.SEEDS["c4"], 0, "c4")
h = job.ts.host()
print("fresh:", job.end_to_end(h)["calls_ms"], flush=True)
stream = torch.cuda.Stream()
with torch.cuda.stream(stream):
    for _ in range(10):
        job.step(stream.cuda_stream)
    torch.cuda.synchronize()
print("after steps on a torch stream:", job.end_to_end(h)["calls_ms"], flush=True)
job.kernel_times(stream, 5)
print("after kernel_times:", job.end_to_end(h)["calls_ms"], flush=True)
import time  # noqa: E402
t0 = time.time()
with torch.cuda.stream(stream):
    while time.time() - t0 < 3.0:
        job.step(stream.cuda_stream)
    torch.cuda.synchronize()
print("after 3 s of staged steps:", job.end_to_end(h)["calls_ms"], flush=True)
m = B.microbench_sustained(25, 8, 20.0, 1.0, 3)
print("after the microbench:", job.end_to_end(h)["calls_ms"], "clock", m[1], flush=True)
time.sleep(2)
print("after 2 s idle:", job.end_to_end(h)["calls_ms"], flush=True)
