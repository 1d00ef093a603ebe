"""Drop-in pipelining A/B on the GPU box: K back-to-back bitcoinconsensus_verify_batch calls over
the C2 inputs for each pipeline chunk size (0 = unpipelined), interleaved over reps, with the
engine's per-call breakdown (bcc_batch_stats) of the best call.

    python tools/e2e_pipe.py [N] [K] [REPS] [chunk ...]        e.g. 1000000 10 2 0 262144 500000
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    chunks = [int(x) for x in sys.argv[4:]] or [0, 262144]
    wl = B.Workload(n, seed=0x5EED0001)
    wl.verify_batch()  # warm
    for rep in range(reps):
        for ch in chunks:
            B.set_pipeline_chunk(ch)
            wl.verify_batch()  # this setting's state
            ms, best = [], None
            c0 = time.process_time()  # CPU time of every thread of the process
            t0 = time.perf_counter()
            for _ in range(k):
                t1 = time.perf_counter()
                nv, _ = wl.verify_batch()
                dt1 = time.perf_counter() - t1
                ms.append(1e3 * dt1)
                if best is None or dt1 < best[0]:
                    best = (dt1, B.last_batch_stats())
                assert nv == n
            dt = time.perf_counter() - t0
            cpu = time.process_time() - c0
            st = best[1]
            rec = dict(chunk=ch, rep=rep, calls=k, sustained_inputs_per_s=round(k * n / dt),
                       best_inputs_per_s=round(n / best[0]), call_ms_min=round(min(ms), 1),
                       call_ms_median=round(sorted(ms)[k // 2], 1),
                       best_breakdown_ms={x: round(st[x + "_seconds"] * 1e3, 2) for x in
                                          ("prepare", "interpret", "stitch", "finish", "stage",
                                           "gpu", "host", "prepare_parse", "prepare_lag",
                                           "process_cpu", "process_cpu_in_gpu_wait")},
                       cpu_ms_per_call=round(1e3 * cpu / k, 1),
                       host_threads=B.host_threads(), cpu_share=B.cpu_share())
            print(json.dumps(rec), flush=True)
    B.set_pipeline_chunk(0)


if __name__ == "__main__":
    main()
