"""bitcoinconsensus_verify_batch from host buffers on the C2 workload (bench.py's drop_in_end_to_end
leg alone): best single call, then `calls` back to back (wall rate and process CPU seconds per 1M
inputs), under the BCC_* environment given (host threads, pipeline chunk, ...)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-bitcoinconsensus_amd"))
if os.environ.get("DROPIN_TORCH"):  # the bench process's setting: torch imported, HIP initialised
    import torch  # noqa: E402
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    if os.environ.get("DROPIN_TORCH") == "stream":
        torch.cuda.set_stream(torch.cuda.Stream())
import bitcoinconsensus_amd as B  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 10
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import host_memory_probe  # noqa: E402
wl = B.Workload(n, seed=0x5EED0001)
wl.run()
best = None
for _ in range(3):
    t0 = time.perf_counter()
    nv, _ = wl.verify_batch()
    dt = time.perf_counter() - t0
    best = dt if best is None else min(best, dt)
    assert nv == n
st = B.last_batch_stats()
mem = host_memory_probe(threads=B.host_threads())
t0, c0 = time.perf_counter(), time.process_time()
for _ in range(calls):
    wl.verify_batch()
sus, cpu = time.perf_counter() - t0, time.process_time() - c0
env = {k: v for k, v in os.environ.items() if k.startswith(("BCC_", "DROPIN_"))}
env["mem_GBps"] = mem
print(f"{env} threads={B.host_threads()} share={B.cpu_share()} one call {n/best/1e6:.1f} M/s | "
      f"sustained {calls*n/sus/1e6:.1f} M/s, {cpu/(calls*n)*1e6:.3f} CPU-s per 1M | "
      f"prepare {st['prepare_seconds']*1e3:.1f} interpret {st['interpret_seconds']*1e3:.1f} ms", flush=True)
if os.environ.get("PHASES"):
    runs = []
    for _ in range(calls):
        wl.verify_batch()
        runs.append(B.last_batch_stats())
    med = lambda k: sorted(r[k] for r in runs)[len(runs) // 2] * 1e3  # noqa: E731
    print("  phases ms: " + " ".join(f"{k.replace('_seconds', '')}={med(k):.2f}" for k in (
        "prepare_seconds", "prepare_parse_seconds", "interpret_seconds", "stage_seconds",
        "stitch_seconds", "finish_seconds", "host_seconds", "gpu_seconds", "total_seconds")) +
        f" cpu/call={med('process_cpu_seconds'):.1f}", flush=True)
def _smaps(key="AnonHugePages"):
    try:
        for ln in open("/proc/self/smaps_rollup"):
            if ln.startswith(key):
                return int(ln.split()[1]) // 1024
    except OSError:
        pass
    return None


print(f"  rss_MiB={_smaps('Rss')} anon_huge_MiB={_smaps()}", flush=True)
if os.environ.get("DUMP"):
    print({k: (round(v * 1e3, 2) if isinstance(v, float) else v) for k, v in st.items()}, flush=True)
