"""Where bench.py's C4 drop-in leg loses time: the same 8M tuples through bcc_pubkey_verify_batch
(bench.TupleJob.end_to_end) before and after the staged TupleSet runs the bench times."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bench  # noqa: E402
import bitcoinconsensus_amd as B  # noqa: E402

job = bench.TupleJob(B, bench.DEFAULT_N["c4"], bench.SEEDS["c4"], 0, "c4")
h = job.ts.host()
job.ts.run()
print("before staged runs:", job.end_to_end(h)["calls_ms"], flush=True)
for _ in range(20):
    job.ts.run()
job.ts.verdicts()
print("after 20 staged runs:", job.end_to_end(h)["calls_ms"], flush=True)
B.release_thread_state()
print("after release_thread_state:", job.end_to_end(h)["calls_ms"], flush=True)
B.microbench_sustained(25, 8, 20.0, 1.0, 3)
print("after microbench_sustained:", job.end_to_end(h)["calls_ms"], flush=True)
