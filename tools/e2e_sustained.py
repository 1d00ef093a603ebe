"""Sustained drop-in rate: K back-to-back bitcoinconsensus_verify_batch calls on the C2 inputs per
host-thread count, with the cgroup's CPU accounting over the whole run (a CFS quota lets a burst
use more CPUs than the quota within one period, but K calls in a row pay for it in throttling).

    python tools/e2e_sustained.py [N] [K] [threads ...]        e.g. 1000000 20 16 32 48 64
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bitcoinconsensus_amd as B  # noqa: E402
from e2e_cgroup import cpu_stat  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    thrs = [int(x) for x in sys.argv[3:]] or [0]
    wl = B.Workload(n, seed=0x5EED0001)
    wl.verify_batch()  # warm
    for rep in range(2):
        for thr in thrs:
            B.set_host_threads(thr)
            wl.verify_batch()  # this thread count's team
            c0 = cpu_stat()
            ms = []
            t0 = time.perf_counter()
            for _ in range(k):
                t1 = time.perf_counter()
                nv, _ = wl.verify_batch()
                ms.append(1e3 * (time.perf_counter() - t1))
                assert nv == n
            dt = time.perf_counter() - t0
            c1 = cpu_stat()
            rec = dict(threads=thr or B.host_threads(), rep=rep, calls=k, total_ms=round(1e3 * dt, 1),
                       inputs_per_s=round(k * n / dt), call_ms_min=round(min(ms), 1),
                       call_ms_median=round(sorted(ms)[k // 2], 1), call_ms_max=round(max(ms), 1))
            for key in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                if key in c0 and key in c1:
                    rec["cg_" + key] = c1[key] - c0[key]
            if "cg_usage_usec" in rec:
                rec["cpus_busy"] = round(rec["cg_usage_usec"] / (1e6 * dt), 2)
            print(json.dumps(rec), flush=True)
    B.set_host_threads(0)


if __name__ == "__main__":
    main()
