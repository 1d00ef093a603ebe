"""Probe: wall time of bitcoinconsensus_verify_batch on the C3 workload vs the engine's own
breakdown (bcc_last_batch_stats)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

shape = [tuple(t) for t in json.load(open(os.path.join(ROOT, "tests", "golden", "block413567_shape.json")))["txs"]]
ntx = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
txs = (shape * (ntx // len(shape) + 1))[:ntx]
wl = B.Workload(kind="block", shape=txs, seed=0x5EED0003)
L = B.blib()
cnt = ctypes.c_size_t(0)
items = L.bcc_workload_items(wl.h, ctypes.byref(cnt))
ret = (ctypes.c_int * cnt.value)()
for _ in range(3):
    L.bitcoinconsensus_verify_batch(items, cnt.value, B.VERIFY_ALL, ret, None)
for _ in range(5):
    t0 = time.perf_counter()
    rc = L.bitcoinconsensus_verify_batch(items, cnt.value, B.VERIFY_ALL, ret, None)
    t1 = time.perf_counter()
    st = B.last_batch_stats()
    print(f"items {cnt.value} valid {rc} wall {1e3 * (t1 - t0):.2f} ms | host {1e3 * st['host_seconds']:.2f} "
          f"gpu {1e3 * st['gpu_seconds']:.2f} prep {1e3 * st['prepare_seconds']:.2f} "
          f"interp {1e3 * st['interpret_seconds']:.2f} merge {1e3 * st['merge_seconds']:.2f} "
          f"stage {1e3 * st['stage_seconds']:.2f} total {1e3 * st['total_seconds']:.2f}", flush=True)
