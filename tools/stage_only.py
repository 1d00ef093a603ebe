"""The ECDSA stage alone on one C2 workload, `reps` times back to back (for a kernel trace of
its timeline: tools/stage_timeline.py).
  python3 tools/stage_only.py [n] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
torch.cuda.set_device(0)
st = torch.cuda.Stream()
wl = B.Workload(n, seed=0x5EED0001)
wl.run(st.cuda_stream)
torch.cuda.synchronize()
for _ in range(reps):
    wl.run_ecdsa(st.cuda_stream)
    torch.cuda.synchronize()
print("ok", n, reps)
