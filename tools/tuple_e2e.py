"""bcc_pubkey_verify_batch from host buffers on the C4 tuple set (bench.py's drop_in_end_to_end leg
alone): best of `reps` calls, with BCC_TUPLE_* environment settings for round-size experiments."""
import ctypes
import os
import sys
import time

import numpy as np

if os.environ.get("WITH_TORCH"):  # bench.py's process: torch imported and its HIP context up
    import torch
    torch.cuda.init()
    torch.zeros(1, device="cuda")

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ts = B.TupleSet(n, kind="c4", seed=0x5EED0004)
h = ts.host()
L = B.lib()
u64p = ctypes.POINTER(ctypes.c_uint64)
L.bcc_pubkey_verify_batch.argtypes = [ctypes.c_void_p, u64p, ctypes.c_void_p, ctypes.c_void_p, u64p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
out = np.zeros(n, np.uint8)
ts_ = []
for _ in range(reps):
    t0 = time.perf_counter()
    rc = L.bcc_pubkey_verify_batch(h["pub_blob"].ctypes.data, h["pub_off"].ctypes.data_as(u64p),
                                   h["msg32"].ctypes.data, h["sig_blob"].ctypes.data,
                                   h["sig_off"].ctypes.data_as(u64p), out.ctypes.data, n, 0)
    ts_.append(time.perf_counter() - t0)
    assert rc == 0
bad = int((out != h["expect"]).sum())
env = {k: v for k, v in os.environ.items() if k.startswith("BCC_TUPLE")}
print(f"{env} n={n} best {min(ts_)*1e3:.1f} ms = {n/min(ts_)/1e6:.1f} M/s, all {[round(t*1e3,1) for t in ts_]}, mismatches {bad}", flush=True)
