"""Drop-in A/B inside ONE process: settings alternate call by call (the box's state drifts
between processes far more than between neighbouring calls), medians per setting.
    python tools/dropin_interleave.py N CALLS_PER_SETTING "chunk:tail[:shards_per_worker[:fused[:direct[:host_threads[:pre_upload]]]]]" ...
"""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

n, calls = int(sys.argv[1]), int(sys.argv[2])
settings = [tuple(int(x) for x in a.split(":")) for a in sys.argv[3:]]
L = B.lib()
L.bcc_set_pipeline_chunk.argtypes = [ctypes.c_size_t]
L.bcc_set_pipeline_tail.argtypes = [ctypes.c_size_t]
L.bcc_set_long_shards_per_worker.argtypes = [ctypes.c_uint]
L.bcc_set_fused_pass.argtypes = [ctypes.c_int]
L.bcc_set_direct_upload.argtypes = [ctypes.c_int]
L.bcc_set_pre_upload.argtypes = [ctypes.c_int]
wl = B.Workload(n, seed=0x5EED0001)
wl.run()
for _ in range(2):
    wl.verify_batch()
res = {s: [] for s in settings}
cpu = {s: [] for s in settings}
stage = {s: [] for s in settings}
host = {s: [] for s in settings}
for k in range(calls):
    for s in settings:
        L.bcc_set_pipeline_chunk(s[0])
        L.bcc_set_pipeline_tail(s[1])
        L.bcc_set_long_shards_per_worker(s[2] if len(s) > 2 else 1)
        L.bcc_set_fused_pass(s[3] if len(s) > 3 else 1)
        L.bcc_set_direct_upload(s[4] if len(s) > 4 else 1)
        B.set_host_threads(s[5] if len(s) > 5 else 0)
        L.bcc_set_pre_upload(s[6] if len(s) > 6 else 1)
        c0, t0 = time.process_time(), time.perf_counter()
        nv, _ = wl.verify_batch()
        res[s].append(time.perf_counter() - t0)
        cpu[s].append(time.process_time() - c0)
        assert nv == n
        st = B.last_batch_stats()
        stage[s].append(st["stage_seconds"])
        host[s].append(st["host_seconds"])
for s in settings:
    m = statistics.median(res[s])
    print(f"chunk {s[0]:>7} tail {s[1]:>7} spw {s[2] if len(s) > 2 else 1} fused {s[3] if len(s) > 3 else 1} "
          f"direct {s[4] if len(s) > 4 else 1} threads {s[5] if len(s) > 5 else 0} pre {s[6] if len(s) > 6 else 1}: median {m * 1e3:6.2f} ms = {n / m / 1e6:5.1f} M/s, "
          f"mean {n / statistics.mean(res[s]) / 1e6:5.1f} M/s, cpu {statistics.median(cpu[s]) / n * 1e6:.3f} "
          f"CPU-s/1M, stage {statistics.median(stage[s]) * 1e3:.2f} ms, host {statistics.median(host[s]) * 1e3:.2f} ms",
          flush=True)
