"""Drop-in end-to-end A/B: bitcoinconsensus_verify_batch on the C2 inputs (1M P2WPKH spends from
host buffers) at several pipeline chunk sizes, interleaved, best of 3 each.
    python tools/e2e_ab.py [N] [chunk ...]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
chunks = [int(x) for x in sys.argv[2:]] or [0, 1 << 17, 1 << 18, 1 << 19]
wl = B.Workload(n, seed=0x5EED0001)
L = B.lib()
L.bcc_set_pipeline_chunk.argtypes = [ctypes.c_size_t]
wl.verify_batch()
res = {c: [] for c in chunks}
for rep in range(3):
    for c in chunks:
        L.bcc_set_pipeline_chunk(c)
        t0 = time.perf_counter()
        nv, _ = wl.verify_batch()
        dt = time.perf_counter() - t0
        st = B.last_batch_stats()
        res[c].append(dict(ms=round(1e3 * dt, 1), valid=nv, host_ms=round(1e3 * st["host_seconds"], 1),
                           gpu_wait_ms=round(1e3 * st["gpu_seconds"], 1),
                           prepare_ms=round(1e3 * st["prepare_seconds"], 1),
                           interpret_ms=round(1e3 * st["interpret_seconds"], 1),
                           stage_ms=round(1e3 * st["stage_seconds"], 1), rounds=st["rounds"]))
        print(json.dumps(dict(chunk=c, rep=rep, **res[c][-1])), flush=True)
for c in chunks:
    best = min(r["ms"] for r in res[c])
    print(json.dumps(dict(chunk=c, best_ms=best, inputs_per_s=round(n / best * 1e3))), flush=True)
L.bcc_set_pipeline_chunk(0)
