"""ECDSA stage time against batch size in residency rounds (R = CUs x 4 SIMDs x 4 waves x 64 lanes):
C2 workloads of n = k*R and the 1M headline, C4 tuple sets at 1M and 8M, each stage timed with HIP
events over `reps` back-to-back runs on one stream.  Run under rocprofv3 --kernel-trace to split
the stage per kernel launch.
  python3 tools/keyq_sweep.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.cuda.set_device(0)
st = torch.cuda.Stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
R = cus * 4 * 4 * 64


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


sizes = [R, 2 * R, 3 * R, 1_000_000, 4 * R, 8 * R, 16 * R]
for n in sizes:
    wl = B.Workload(n, seed=0x5EED0001)
    wl.run(st.cuda_stream)
    torch.cuda.synchronize()
    ms = timed(lambda: wl.run_ecdsa(st.cuda_stream))
    print(f"c2 n={n:9d} rounds={n / R:6.3f} stage {ms:7.3f} ms  per 1M {ms * 1e6 / n:6.3f} ms  "
          f"per round {ms * R / n:6.3f} ms", flush=True)
    del wl
for n in (1_000_000, 8_000_000):
    ts = B.TupleSet(n, seed=0x5EED0004)
    ms = timed(lambda: ts.run(st.cuda_stream))
    print(f"c4 n={n:9d} rounds={n / R:6.3f} run   {ms:7.3f} ms  per 1M {ms * 1e6 / n:6.3f} ms", flush=True)
    del ts
