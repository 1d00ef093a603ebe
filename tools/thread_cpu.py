"""Per-thread CPU time of the process over K back-to-back C2 drop-in calls (GPU box): which
threads burn the CPU quota -- the engine's teams, the pipeline worker, or the HIP runtime's own.

    python tools/thread_cpu.py [N] [K] [chunk]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402

TICK = os.sysconf("SC_CLK_TCK")


def threads():
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            comm = open(f"/proc/self/task/{tid}/comm").read().strip()
            f = open(f"/proc/self/task/{tid}/stat").read().rsplit(")", 1)[1].split()
            out[int(tid)] = (comm, (int(f[11]) + int(f[12])) / TICK)
        except OSError:
            pass
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 500000
    B.set_pipeline_chunk(chunk)
    wl = B.Workload(n, seed=0x5EED0001)
    for _ in range(3):
        wl.verify_batch()
    a = threads()
    c0, t0 = time.process_time(), time.perf_counter()
    for _ in range(k):
        wl.verify_batch()
    dt, cpu = time.perf_counter() - t0, time.process_time() - c0
    b = threads()
    per = {}
    for tid, (comm, s) in b.items():
        d = s - a.get(tid, (comm, 0.0))[1]
        key = comm
        per.setdefault(key, [0.0, 0])
        per[key][0] += d
        per[key][1] += 1
    print(f"chunk {chunk}: {k} calls, {k * n / dt / 1e6:.2f} M inputs/s, process CPU {1e3 * cpu / k:.1f} ms per call")
    for comm, (s, cnt) in sorted(per.items(), key=lambda x: -x[1][0])[:12]:
        print(f"  {comm:20s} threads {cnt:3d}  CPU {1e3 * s / k:8.1f} ms per call")
    # every thread (the engine's are unnamed): the main thread first, then by CPU
    me = os.getpid()
    rows = sorted(((tid, b[tid][1] - a.get(tid, ("", 0.0))[1]) for tid in b), key=lambda x: -x[1])
    print("  per thread (ms per call, tid - pid):",
          " ".join(f"{tid - me}:{1e3 * d / k:.1f}" for tid, d in rows if d > 0))


if __name__ == "__main__":
    main()
