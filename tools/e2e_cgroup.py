"""Drop-in end to end (bitcoinconsensus_verify_batch on the C2 inputs from host buffers) with the
process's CPU accounting around every call: the cgroup's cpu.stat (usage, nr_throttled,
throttled_usec) and getrusage (page faults, context switches, user / system time), for several
(pipeline chunk, host threads) configurations, interleaved, 3 calls each.

    python tools/e2e_cgroup.py [N] [chunk:threads ...]     e.g. 0:16 262144:16 262144:12
"""
import json
import os
import resource
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bitcoinconsensus_amd as B  # noqa: E402


def cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if len(ln.split()) == 2)}
    except OSError:
        return {}


def ru():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return dict(minflt=r.ru_minflt, majflt=r.ru_majflt, nvcsw=r.ru_nvcsw, nivcsw=r.ru_nivcsw,
                utime=r.ru_utime, stime=r.ru_stime)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    cfgs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]] or [(0, 0), (262144, 0)]
    try:
        cpu_max = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        cpu_max = None
    print(json.dumps(dict(n=n, cpu_share=B.cpu_share(), default_host_threads=B.host_threads(),
                          cpu_max=cpu_max, affinity=len(os.sched_getaffinity(0)),
                          nproc=os.cpu_count())), flush=True)
    wl = B.Workload(n, seed=0x5EED0001)
    wl.verify_batch()  # warm: device tables, pinned buffers, thread state
    best = {}
    for rep in range(3):
        for chunk, thr in cfgs:
            B.set_pipeline_chunk(chunk)
            B.set_host_threads(thr)
            c0, r0 = cpu_stat(), ru()
            t0 = time.perf_counter()
            nv, _ = wl.verify_batch()
            dt = time.perf_counter() - t0
            c1, r1 = cpu_stat(), ru()
            st = B.last_batch_stats()
            rec = dict(chunk=chunk, threads=thr or B.host_threads(), rep=rep, ms=round(1e3 * dt, 1),
                       valid=nv, rounds=st["rounds"],
                       host_ms=round(1e3 * st["host_seconds"], 1),
                       gpu_wait_ms=round(1e3 * st["gpu_seconds"], 1),
                       prepare_ms=round(1e3 * st["prepare_seconds"], 1),
                       interpret_ms=round(1e3 * st["interpret_seconds"], 1),
                       stage_ms=round(1e3 * st["stage_seconds"], 1),
                       shard_ms=round(1e3 * st["shard_seconds"], 1),
                       stitch_ms=round(1e3 * st["stitch_seconds"], 1),
                       finish_ms=round(1e3 * st["finish_seconds"], 1),
                       host_jobs_ms=round(1e3 * st["host_jobs_seconds"], 1),
                       prep_lag_ms=round(1e3 * st["prepare_lag_seconds"], 2),
                       prep_parse_ms=round(1e3 * st["prepare_parse_seconds"], 2),
                       prep_hash_ms=round(1e3 * st["prepare_hash_seconds"], 2))
            for k in ("usage_usec", "user_usec", "system_usec", "nr_periods", "nr_throttled",
                      "throttled_usec"):
                if k in c0 and k in c1:
                    rec["cg_" + k] = c1[k] - c0[k]
            for k in r0:
                rec["ru_" + k] = round(r1[k] - r0[k], 4)
            if "cg_usage_usec" in rec:
                rec["cpus_busy"] = round(rec["cg_usage_usec"] / (1e6 * dt), 2)
            print(json.dumps(rec), flush=True)
            key = (chunk, thr)
            best[key] = min(best.get(key, 1e9), dt)
    for (chunk, thr), dt in best.items():
        print(json.dumps(dict(chunk=chunk, threads=thr, best_ms=round(1e3 * dt, 1),
                              inputs_per_s=round(n / dt))), flush=True)
    B.set_pipeline_chunk(0)
    B.set_host_threads(0)


if __name__ == "__main__":
    main()
