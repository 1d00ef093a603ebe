"""Probe: bitcoinconsensus_verify_batch end to end (host buffers) on the C2 workload, with the
engine's own breakdown.  python tools/e2e_probe.py [N]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
wl = B.Workload(n, seed=0x5EED0001)
L = B.blib()
cnt = ctypes.c_size_t(0)
items = L.bcc_workload_items(wl.h, ctypes.byref(cnt))
ret = (ctypes.c_int * cnt.value)()
L.bitcoinconsensus_verify_batch(items, cnt.value, B.VERIFY_ALL, ret, None)
for _ in range(3):
    t0 = time.perf_counter()
    rc = L.bitcoinconsensus_verify_batch(items, cnt.value, B.VERIFY_ALL, ret, None)
    t1 = time.perf_counter()
    st = B.last_batch_stats()
    print(f"items {cnt.value} valid {rc} wall {1e3 * (t1 - t0):.1f} ms ({cnt.value / (t1 - t0) / 1e6:.2f} M/s) | "
          + " ".join(f"{k.replace('_seconds', '')} {1e3 * st[k]:.1f}" for k in st if k.endswith("seconds")),
          flush=True)
