"""bench.py — ECDSA verifies/s of the MI355X signature hot path (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --config c2|c3|c4|c5|c5t --n UNITS_PER_GPU]
    (N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
             --master-port P bench.py --gpus N ...)

Default workload (BASELINE.json configs[1]): n synthetic P2WPKH spends per GPU
(default 1,000,000), inputs resident in HBM (staged by the engine's own first-round interpreter
pass).  One step = one pass of the hot path over the batch: BIP143 sighash kernels (aux hashes,
patch, preimage SHA-256d) + the ECDSA kernels (batched s^-1, pubkey decompression + GLV + Q table,
Strauss ladder + x-check).  value = verifies of all ranks / max-over-ranks wall time of K steps.
Multi-GPU is weak scaling: the N ranks partition ONE global input set of N x n units from the
config's seed (rank r takes units [r n, (r + 1) n)), no collective in the timed
loop; afterwards the validity bitmaps are all-gathered over RCCL and checked.

Other configs (run explicitly, results committed under profiles/):
  c3  block replay: transactions shaped like the reference's bench block413567 (tiled to 4,000
      txs), mixed P2PKH / P2WPKH / P2SH 2-of-3, through bitcoinconsensus_verify_batch end to end
      (host buffers -> threaded host interpreter -> GPU sighash + ECDSA rounds -> verdicts); a
      step is one verify_batch call.
  c4  ECDSA tuples (pub, msg32, DER sig), 90 % valid + 18 adversarial classes, staged rows in HBM
      (8M per GPU = the per-GPU shard of the 64M-tuple node batch); a step is the ECDSA kernels.
  c5  BIP340 rows (GPU-signed + the 15 BIP340 vectors tiled), a step is the Schnorr kernels.

Also reported:
  roofline      the signature kernels against the measured v_mad_u64_u32 issue rate (int-ALU
                bound: MFMA is deliberately unused; SURVEY.md §8d W = 2,257 modmuls = 144,448
                32x32->64 partial products per ECDSA verify; DESIGN.md §3 for BIP340), kernel time
                from HIP events on the launch stream
  cpu_baseline  the REFERENCE (oracle/_ref: Bitcoin Core v0.21 libbitcoinconsensus + libsecp256k1
                built from /root/reference) on a bounded sample of the same inputs, std::thread
                pool over the host cores (rank 0, N = 1 only)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))

MADS_PER_VERIFY = 144448          # 2,257 modmuls x 64 (32x32->64) products
MADS_PER_SCHNORR = 142848         # 2,232 modmuls x 64
METRIC = "ECDSA verifies/sec (node) at 1/2/4/8 MI355X; % of int-ALU roofline"
DEFAULT_N = {"c2": 1_000_000, "c3": 4000, "c4": 8_000_000, "c5": 16_000_000, "c5t": 1_000_000}
SEEDS = {"c2": 0x5EED0001, "c3": 0x5EED0003, "c4": 0x5EED0004, "c5": 0x5EED0005,
         "c5t": 0x5EED0006}
# the ECDSA stage's kernels (the square-root-free twist path)
ECDSA_KERNELS = ("ecdsa (batch_sinv + twist_keyq + twist_ladder_g + twist_fin<ecdsa>; "
                 "no key square root)")
SCHNORR_KERNELS = ("schnorr (schnorr_tladder: prep + ladder fused, + twist_fin<bip340>; "
                   "no lift_x square root)")
CPU_PASSES = 3                    # timed passes of the CPU baseline (median), after 1 warm-up


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _reference():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_ctypes import Reference, reference_available
    return Reference() if reference_available() else None


def host_cpu_info():
    """CPU model, logical / physical counts and the threads the baseline uses: the smaller of the
    affinity mask and the cgroup CPU quota (on a shared GPU box os.cpu_count() shows the whole
    machine, the quota is the share this process may use).  BASELINE.md §3: rayon's default is
    one worker per logical CPU the process can run on."""
    info = {"logical_cpus_visible": os.cpu_count()}
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    info["affinity_cpus"] = aff
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(round(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    model, cores = None, set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
            elif not k and phys is not None:
                cores.add((phys, core))
                phys = core = None
    except OSError:
        pass
    info["model"] = model
    info["physical_cores_visible"] = len(cores) or None
    info["threads_used"] = min(aff, quota) if quota else aff
    return info


def newest_cost_model():
    """The ladder's instruction-class decomposition of the newest round that committed one
    (profiles/rNN/ladder_cost_model.json, tools/isa/cost_model.py)."""
    import glob
    import re
    found = [(int(re.search(r"/r(\d+)/", c).group(1)), c)
             for c in glob.glob(os.path.join(ROOT, "profiles", "r*", "ladder_cost_model.json"))
             if re.search(r"/r(\d+)/", c)]
    return max(found)[1] if found else ""


def _proc_stat_busy():
    """(busy, total) jiffies over all CPUs of the machine (/proc/stat 'cpu' line)."""
    try:
        f = [int(x) for x in open("/proc/stat").readline().split()[1:]]
    except (OSError, ValueError):
        return None
    idle = f[3] + (f[4] if len(f) > 4 else 0)
    return sum(f) - idle, sum(f)


def _cpu_topology():
    """cpu -> (numa node, physical core key) from sysfs (empty when unavailable)."""
    import glob
    topo = {}
    for nd in glob.glob("/sys/devices/system/node/node[0-9]*"):
        node = int(nd.rsplit("node", 1)[1])
        try:
            spec = open(os.path.join(nd, "cpulist")).read().strip()
        except OSError:
            continue
        for part in spec.split(","):
            if not part:
                continue
            a, _, b = part.partition("-")
            for c in range(int(a), int(b or a) + 1):
                topo[c] = [node, None]
    for c in list(topo):
        try:
            sib = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
            topo[c][1] = sib
        except OSError:
            pass
    return topo


def _thread_cpus():
    """{tid: (last cpu, utime+stime jiffies)} of this process's threads (/proc/self/task)."""
    out = {}
    try:
        tids = os.listdir("/proc/self/task")
    except OSError:
        return out
    for t in tids:
        try:
            f = open(f"/proc/self/task/{t}/stat").read().rsplit(")", 1)[1].split()
            out[int(t)] = (int(f[36]), int(f[11]) + int(f[12]))
        except (OSError, ValueError, IndexError):
            pass
    return out


def _smaps_mib():
    """This process's resident and transparent-huge-page memory (MiB, /proc/self/smaps_rollup)."""
    out = {}
    try:
        for ln in open("/proc/self/smaps_rollup"):
            k = ln.split(":")[0]
            if k in ("Rss", "AnonHugePages"):
                out[k] = int(ln.split()[1]) // 1024
    except (OSError, ValueError, IndexError):
        pass
    try:
        out["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
    except OSError:
        pass
    return out


def host_memory_probe(threads=16, mib=64, reps=4):
    """Aggregate host copy bandwidth (GB/s, read + write) of `threads` threads each copying its own
    `mib` MiB buffer `reps` times (numpy copies release the GIL): the memory-side state of the
    shared host at the moment the drop-in leg runs (its host pass is memory-heavy)."""
    import threading
    import numpy as np
    bufs = [(np.ones(mib << 20, np.uint8), np.empty(mib << 20, np.uint8)) for _ in range(threads)]
    for a, b in bufs:
        np.copyto(b, a)  # fault in

    def work(a, b):
        for _ in range(reps):
            np.copyto(b, a)
    ts = [threading.Thread(target=work, args=ab) for ab in bufs]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt = time.perf_counter() - t0
    return round(2 * threads * reps * (mib << 20) / dt / 1e9, 1)


def gpu_numa_node(dev):
    """NUMA node of GPU `dev` (sysfs of its PCI function; None when unknown)."""
    try:
        import torch
        bus = torch.cuda.get_device_properties(dev).pci_bus_id
        dom = getattr(torch.cuda.get_device_properties(dev), "pci_domain_id", 0)
        for cand in (f"/sys/bus/pci/devices/{dom:04x}:{bus:02x}:00.0/numa_node",):
            if os.path.exists(cand):
                return int(open(cand).read())
    except Exception:  # noqa: BLE001 (diagnostic only)
        pass
    return None


def host_placement(before, after, topo):
    """Where the call's busy threads ran: the CPUs (and NUMA nodes / distinct physical cores) of
    the threads that used CPU time between two _thread_cpus() snapshots."""
    busy = {t: (c, j - before.get(t, (c, 0))[1]) for t, (c, j) in after.items()}
    busy = {t: v for t, v in busy.items() if v[1] > 0}
    cpus = sorted({c for c, _ in busy.values()})
    nodes = {}
    for c in cpus:
        n = topo.get(c, [None])[0]
        nodes[str(n)] = nodes.get(str(n), 0) + 1
    cores = {topo[c][1] for c in cpus if c in topo and topo[c][1]}
    return dict(busy_threads=len(busy), cpus=cpus, cpus_per_numa_node=nodes,
                distinct_physical_cores=len(cores) or None)


def median_rate(run, n, passes=CPU_PASSES):
    """1 warm-up + `passes` timed runs of run() (returns seconds); median items/s and all passes."""
    run()
    secs = sorted(run() for _ in range(passes))
    return n / secs[len(secs) // 2], [round(n / s, 1) for s in secs]


def cpu_baseline_script(items, what, unit="inputs/s", gpu_verdicts=None):
    """Reference libbitcoinconsensus over (spk, amount, tx, nin) items (checker-side code):
    bitcoinconsensus_verify_script_with_amount per item on a dynamically chunked std::thread
    pool (oracle/ref_shim.cpp), median of CPU_PASSES passes; the single-core rate beside it.
    gpu_verdicts: the GPU's per-item verdicts on the same items (0/1 bytes) -> mismatch count."""
    import ctypes
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_consensus.so")
    if not os.path.exists(ref):
        return None
    L = ctypes.CDLL(ref)
    L.ref_bench_verify_script.restype = ctypes.c_double
    sample = len(items)
    hw = host_cpu_info()
    threads = hw["threads_used"]

    def blob(parts):
        off = [0]
        for p in parts:
            off.append(off[-1] + len(p))
        return b"".join(parts), (ctypes.c_long * len(off))(*off)

    sb, so = blob([it[0] for it in items])
    tb, to = blob([it[2] for it in items])
    am = (ctypes.c_int64 * sample)(*[it[1] for it in items])
    nin = (ctypes.c_uint * sample)(*[it[3] for it in items])
    ret = (ctypes.c_int * sample)()
    args = (sb, so, tb, to, am, nin, ctypes.c_uint(0xE15), ret)
    rate, passes = median_rate(
        lambda: L.ref_bench_verify_script(ctypes.c_int(threads), ctypes.c_long(sample), *args),
        sample)
    ok = sum(ret[i] for i in range(sample))
    n1 = max(1, sample // 16)
    rate1, _ = median_rate(
        lambda: L.ref_bench_verify_script(ctypes.c_int(1), ctypes.c_long(n1), *args), n1, passes=1)
    mism = None
    if gpu_verdicts is not None:
        mism = sum(1 for i in range(sample) if (ret[i] == 1) != (gpu_verdicts[i] == 1))
    return dict(value=rate, unit=unit, cores=threads, kind="reference",
                sample=f"{sample} {what}, bitcoinconsensus_verify_script_with_amount flags=0xE15, "
                       f"dynamically chunked std::thread pool x{threads}, median of "
                       f"{CPU_PASSES} passes after 1 warm-up; reference accepted {ok}/{sample}"
                       + ("" if mism is None else f"; GPU verdict mismatches on the sample: {mism}"),
                passes=passes, single_core_value=rate1, host=hw,
                gpu_verdict_mismatches=mism)


def aggregate(elapsed, n_valid, world, device="cuda"):
    """Max of the per-rank timed wall clocks and the sum of valid verdicts over all ranks.
    The only collectives of a bench run; they sit outside the timed region."""
    if world <= 1:
        return elapsed, n_valid
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([n_valid], device=device, dtype=torch.int64)
    dist.all_reduce(c)
    return t.item(), int(c.item())


def gather_verdicts(local, world, device="cuda"):
    """All-gather every rank's verdicts as packed validity bitmaps (1 bit per input) and return
    the global verdict array in rank order.  The only data collective of a sharded run (SURVEY.md
    §8e: RCCL all_gather on the GPUs, gloo in the CPU tests); it sits outside the timed loop."""
    import numpy as np
    local = np.asarray(local, dtype=np.uint8)
    if world <= 1:
        return local
    import torch
    import torch.distributed as dist
    n = torch.tensor([len(local)], device=device, dtype=torch.int64)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    nbytes = (max(ns) + 7) // 8
    bits = np.zeros(nbytes, np.uint8)
    pk = np.packbits(local)
    bits[: len(pk)] = pk
    t = torch.from_numpy(bits).to(device)
    out = torch.empty(world * nbytes, dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, t)
    allb = out.cpu().numpy().reshape(world, nbytes)
    return np.concatenate([np.unpackbits(allb[r])[: ns[r]] for r in range(world)])


def c1_vector():
    """Config C1: the README P2PKH spend (lib.rs:223-231), as committed in crate_vectors.json."""
    v = next(x for x in json.load(open(os.path.join(ROOT, "tests", "golden", "crate_vectors.json")))
             if x["name"] == "p2pkh")
    return bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"], v["flags"]


def single_call_latency(B, calls=200):
    """Latency of ONE bitcoinconsensus_verify_script_with_amount call on C1 (what an unchanged Rust
    caller of verify() sees, lib.rs:103-139): its round on the GPU (bcc_set_host_small_round(0)),
    and the default, which verifies rounds of <= 16 checks with the engine's host code."""
    import statistics
    spk, amount, tx, nin, flags = c1_vector()

    def lat():
        ts = []
        for _ in range(calls):
            t0 = time.perf_counter()
            r = B.verify_script_with_amount(spk, amount, tx, nin, flags)
            ts.append(time.perf_counter() - t0)
            assert r == (1, 0)
        return statistics.median(ts) * 1e6
    B.set_host_small_round(0)  # every round on the GPU
    try:
        B.verify_script_with_amount(spk, amount, tx, nin, flags)  # warm
        gpu_us = lat()
    finally:
        B.set_host_small_round(B.HOST_SMALL_ROUND_DEFAULT)  # the default: small rounds on the host
    B.verify_script_with_amount(spk, amount, tx, nin, flags)
    host_us = lat()
    return dict(config="C1: README P2PKH tx, input 0", calls=calls, gpu_round_us=gpu_us,
                host_small_round_us=host_us,
                note="median per-call latency; the reference's own per-call latency is in "
                     "cpu_baseline.single_call_us")


# ---- per-config jobs: stage inputs, run one step, time the dominant kernels, CPU baseline ----

class C2:
    unit = "verifies/s"

    def __init__(self, B, n, seed, dev, first=0, total=None):
        self.B = B
        self.dev = dev
        self.wl = B.Workload(n, seed=seed, device=dev, first=first)
        self.shape = self.wl.shape()
        self.units = self.shape["tuples"]
        self.n = n

    def step(self, sp):
        self.wl.run(sp)

    def valid(self):
        return sum(self.wl.verdicts())

    def item_verdicts(self):
        v = self.wl.verdicts()
        out = bytearray(self.n)
        for t, i in enumerate(self.wl.tuple_items()):
            out[i] = v[t]
        return out

    def kernel_times(self, stream, reps):
        import torch
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        sp = stream.cuda_stream
        e[0].record(stream)
        for _ in range(reps):
            self.wl.run_sighash(sp)
        e[1].record(stream)
        for _ in range(reps):
            self.wl.run_ecdsa(sp)
        e[2].record(stream)
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]) / reps, e[1].elapsed_time(e[2]) / reps

    def extra(self, sighash_ms):
        sh = self.shape
        b = sh["sighash_bytes"]
        out = {"sighash_stage": dict(kernels="sha256d aux/legacy templates + BIP143 from raw tx bytes "
                                             "(K_wtx parse + per-tx hashes, K_win preimage) + patch + "
                                             "sha256d preimages",
                                     avg_ms=sighash_ms, algorithmic_bytes=b,
                                     achieved_GBps=b / (sighash_ms * 1e-3) / 1e9, peak_GBps=8000.0)}
        if type(self) is C2:
            out["drop_in_end_to_end"] = self.end_to_end()
            out["single_call"] = single_call_latency(self.B)
        return out

    def end_to_end(self, reps=3, calls=20):
        """The same inputs through bitcoinconsensus_verify_batch from host buffers (deserialize,
        interpreter, sighash jobs, H2D, kernels, verdicts back): what a drop-in caller sees.
        Reported beside value, never as value (inputs are not HBM-resident).  Also the host phase
        split (bcc_batch_stats, median per field over the sustained calls), the process CPU time
        per call, where the host threads ran (CPUs, NUMA nodes, physical cores vs the GPU's node)
        and how busy the whole machine was meanwhile (other tenants share its cores)."""
        import statistics
        best, st = None, None
        for _ in range(reps):
            t0 = time.perf_counter()
            nv, _ = self.wl.verify_batch()
            dt = time.perf_counter() - t0
            if best is None or dt < best:
                best, st = dt, self.B.last_batch_stats()
        # sustained: calls back to back (a CFS CPU quota lets one call burst above it, a run of
        # calls pays for that in throttling), whole-run wall time
        runs = []
        mem_probe = host_memory_probe(threads=self.B.host_threads())
        topo = _cpu_topology()
        th0, ps0 = _thread_cpus(), _proc_stat_busy()
        t0, c0 = time.perf_counter(), time.process_time()
        for _ in range(calls):
            self.wl.verify_batch()
            runs.append(self.B.last_batch_stats())
        sus, cpu_s = time.perf_counter() - t0, time.process_time() - c0
        th1, ps1 = _thread_cpus(), _proc_stat_busy()
        med = lambda k: statistics.median(r[k] for r in runs)  # noqa: E731
        ms = lambda k: round(med(k) * 1e3, 3)  # noqa: E731
        phases = dict(prepare_ms=ms("prepare_seconds"), prepare_parse_ms=ms("prepare_parse_seconds"),
                      prepare_hash_ms=ms("prepare_hash_seconds"),
                      interpret_ms=ms("interpret_seconds"), stage_ms=ms("stage_seconds"),
                      stitch_ms=ms("stitch_seconds"), finish_ms=ms("finish_seconds"),
                      host_ms=ms("host_seconds"), gpu_wait_ms=ms("gpu_seconds"),
                      total_ms=ms("total_seconds"),
                      process_cpu_s_per_call=round(med("process_cpu_seconds"), 4),
                      process_cpu_in_gpu_wait_s=round(med("process_cpu_in_gpu_wait_seconds"), 4),
                      rounds=med("rounds"),
                      note=f"median per field over the {calls} sustained calls (bcc_batch_stats); "
                           "the host phases of pipelined chunks overlap their device rounds")
        machine = None
        if ps0 and ps1 and ps1[1] > ps0[1]:
            machine = dict(busy_fraction_all_cpus=round((ps1[0] - ps0[0]) / (ps1[1] - ps0[1]), 3),
                           logical_cpus=os.cpu_count(),
                           loadavg=open("/proc/loadavg").read().split()[:3]
                           if os.path.exists("/proc/loadavg") else None,
                           note="whole machine over the sustained calls, this process included")
        machine = dict(machine or {}, host_copy_GBps=mem_probe,
                       host_copy_note="host_memory_probe: host_threads threads x 64 MiB numpy "
                                      "copies, read + write bytes, just before the sustained calls")
        place = host_placement(th0, th1, topo)
        place["process_memory_MiB"] = _smaps_mib()
        place["gpu_numa_node"] = gpu_numa_node(getattr(self, "dev", 0))
        return dict(inputs_per_s=self.n / best, ms=best * 1e3, valid=nv,
                    host_ms=st["host_seconds"] * 1e3, gpu_ms=st["gpu_seconds"] * 1e3,
                    h2d_ms=st["stage_seconds"] * 1e3, host_threads=self.B.host_threads(),
                    cpu_share=self.B.cpu_share(), sustained_inputs_per_s=calls * self.n / sus,
                    sustained_calls=calls,
                    # process CPU (every thread) per 1M inputs over the sustained calls
                    sustained_cpu_s_per_M=cpu_s / (calls * self.n) * 1e6,
                    sustained_cpus_busy=cpu_s / sus,
                    phases=phases, host_placement=place, machine=machine)

    def cpu(self, sample):
        sample = min(sample, self.n)
        # per-item GPU verdicts of the benchmarked staged path (one tuple per P2WPKH item)
        v = self.wl.verdicts()
        item_v = bytearray(self.n)
        for t, i in enumerate(self.wl.tuple_items()):
            item_v[i] = v[t]
        cb = cpu_baseline_script([self.wl.item(i) for i in range(sample)],
                                 f"C2 inputs (first {sample} of rank 0's workload)",
                                 unit="verifies/s", gpu_verdicts=item_v[:sample])
        R = _reference()
        if cb is not None and R is not None:
            import statistics
            spk, amount, tx, nin, flags = c1_vector()
            ts = []
            for _ in range(2000):
                t0 = time.perf_counter()
                R.verify_script_with_amount(spk, amount, tx, nin, flags)
                ts.append(time.perf_counter() - t0)
            cb["single_call_us"] = statistics.median(ts) * 1e6
            cb["single_call"] = "C1 README tx, one bitcoinconsensus_verify_script_with_amount call, median of 2000"
        return cb

    def config(self, world):
        return {"workload": "C2: synthetic P2WPKH inputs, BIP143 sighash + ECDSA verify "
                            "(BASELINE.json configs[1])",
                "inputs_per_gpu": self.n, "global_inputs": self.n * world,
                "parallelism": f"shard x{world} (independent tuples, no collective)"}

    data = "synthetic (deterministic P2WPKH spends, GPU-generated keys/signatures)"
    mads = MADS_PER_VERIFY
    kernel = ECDSA_KERNELS


class C3(C2):
    """Block replay through the drop-in batch ABI, end to end from host buffers."""
    unit = "inputs/s"

    def __init__(self, B, n, seed, dev, first=0, total=None):
        self.B = B
        seed += first  # block shards: independent batches (a block's txs stay on one GPU)
        shape = [tuple(t) for t in json.load(open(os.path.join(
            ROOT, "tests", "golden", "block413567_shape.json")))["txs"]]
        txs = (shape * (n // len(shape) + 1))[:n]
        self.ntx = n
        self.wl = B.Workload(kind="block", shape=txs, seed=seed, device=dev)
        self.shape = self.wl.shape()
        self.units = self.wl.n           # inputs
        self.n = self.wl.n
        self._valid = 0

    def step(self, sp):
        self._valid, _ = self.wl.verify_batch()

    def item_verdicts(self):
        return self._ret

    def valid(self):
        self._valid, self._ret = self.wl.verify_batch()
        # per-call host / device breakdown: the median of each field over 21 calls (one call's
        # numbers vary by ±10 % with the box's CPU share)
        runs = [self.B.last_batch_stats()]
        for _ in range(20):
            self.wl.verify_batch()
            runs.append(self.B.last_batch_stats())
        self.stats = {k: sorted(r[k] for r in runs)[len(runs) // 2] for k in runs[0]}
        return self._valid

    def extra(self, sighash_ms):
        e = C2.extra(self, sighash_ms)
        st = self.stats
        e["batch_stats"] = dict(st, note="median over 21 calls per field")
        e["note"] = ("value = inputs/s of bitcoinconsensus_verify_batch end to end from host "
                     "buffers (host deserialize + interpreter + preimage building on up to 16 "
                     "threads, H2D, GPU sighash + ECDSA, re-run rounds for CHECKMULTISIG key "
                     "advance); roofline = the first round's staged ECDSA kernels in HBM")
        return e

    def cpu(self, sample):
        sample = min(sample, self.n)
        _, ret = self.wl.verify_batch()
        return cpu_baseline_script([self.wl.item(i) for i in range(sample)],
                                   f"C3 inputs (first {sample})", gpu_verdicts=ret[:sample])

    def config(self, world):
        return {"workload": f"C3: block replay, {self.ntx} txs with block413567's input/output "
                            "histogram, 60% P2PKH / 30% P2WPKH / 10% P2SH 2-of-3, "
                            "bitcoinconsensus_verify_batch end to end (BASELINE.json configs[2])",
                "inputs_per_gpu": self.n, "global_inputs": self.n * world,
                "parallelism": f"shard x{world} (independent batches, no collective)"}

    data = "synthetic (block413567-shaped txs re-signed with GPU-generated keys/signatures)"


class TupleJob:
    def __init__(self, B, n, seed, dev, kind, first=0, total=None):
        import bitcoinconsensus_amd as BB
        vec = []
        if kind == "c5":
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            from fixtures import bip340_vectors
            vec = [(t["sig"], t["msg"], t["pub"], t["verdict"]) for t in bip340_vectors()]
        self.kind = kind
        self.dev = dev
        self.ts = BB.TupleSet(n, kind=kind, seed=seed, device=dev, vectors=vec, first=first,
                              total=total)
        self.units = self.n = n
        self.unit = "verifies/s"
        self.mads = MADS_PER_VERIFY if kind == "c4" else MADS_PER_SCHNORR
        self.kernel = (ECDSA_KERNELS if kind == "c4"
                       else SCHNORR_KERNELS)

    def step(self, sp):
        self.ts.run(sp)

    def valid(self):
        import numpy as np
        v = np.frombuffer(self.ts.verdicts(), np.uint8)
        h = self.ts.host()
        self.mismatch_vs_construction = int((v != h["expect"]).sum())
        return int(v.sum())

    def item_verdicts(self):
        return self.ts.verdicts()

    def kernel_times(self, stream, reps):
        import torch
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record(stream)
        for _ in range(reps):
            self.ts.run(stream.cuda_stream)
        e[1].record(stream)
        torch.cuda.synchronize()
        return 0.0, e[0].elapsed_time(e[1]) / reps

    def extra(self, sighash_ms):
        import numpy as np
        h = self.ts.host()
        out = {"expected_valid": int(h["expect"].sum()),
               "mismatch_vs_construction": self.mismatch_vs_construction,
               "class_counts": np.bincount(h["cls"]).tolist()}
        if self.kind == "c4":
            out["drop_in_end_to_end"] = self.end_to_end(h)
            # the late-allocation case: the caller's pinned round images, device
            # batches and scratch released and allocated again by the next call, after the whole
            # run -- its first call pays the allocation, the next ones show whether the late
            # placement itself is slower
            import bitcoinconsensus_amd as BB
            BB.release_thread_state()
            late = self.end_to_end(h, reps=4)
            out["drop_in_late_alloc"] = dict(calls_ms=late["calls_ms"],
                                             verifies_per_s_after_first=self.n / (min(late["calls_ms"][1:]) * 1e-3),
                                             mismatches_vs_staged=late["mismatches_vs_staged"],
                                             note="bcc_release_thread_state() after the timed run, then 4 "
                                                  "calls; the first allocates the thread's state again")
        return out

    def end_to_end(self, h, reps=3):
        """The same n tuples through bcc_pubkey_verify_batch from host buffers: N x
        CPubKey(pub).Verify(hash, sig) (pubkey.cpp:191-207): the caller's blobs copied and uploaded as
        they are, the length filter + lax DER on the device (K_der), kernels, verdicts back.  Reported beside value, never as value."""
        import ctypes
        import numpy as np
        import bitcoinconsensus_amd as BB
        L = BB.lib()
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.bcc_pubkey_verify_batch.argtypes = [ctypes.c_void_p, u64p, ctypes.c_void_p,
                                              ctypes.c_void_p, u64p, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_int]
        out = np.zeros(self.n, np.uint8)
        best, calls = None, []
        for _ in range(reps):  # (the first call of a process allocates the pinned round images)
            t0 = time.perf_counter()
            rc = L.bcc_pubkey_verify_batch(
                h["pub_blob"].ctypes.data, h["pub_off"].ctypes.data_as(u64p), h["msg32"].ctypes.data,
                h["sig_blob"].ctypes.data, h["sig_off"].ctypes.data_as(u64p), out.ctypes.data,
                self.n, self.dev)
            dt = time.perf_counter() - t0
            assert rc == 0
            best = dt if best is None else min(best, dt)
            calls.append(round(dt * 1e3, 2))
        v = np.frombuffer(self.ts.verdicts(), np.uint8)
        return dict(verifies_per_s=self.n / best, ms=best * 1e3, calls_ms=calls,
                    mismatches_vs_staged=int((out != v).sum()),
                    entry="bcc_pubkey_verify_batch (CPubKey::Verify semantics) from host buffers")

    def cpu(self, sample):
        import numpy as np
        R = _reference()
        if R is None:
            return None
        sample = min(sample, self.n)
        h = self.ts.host()
        if self.kind == "c4":
            args = (h["pub_blob"], h["pub_off"], h["msg32"], h["sig_blob"], h["sig_off"])
            f, what = R.pubkey_verify_blob, "CPubKey::Verify"
        else:
            args = (h["sig64"], h["msg32"], h["xonly32"])
            f, what = R.schnorr_verify_rows, "secp256k1_schnorrsig_verify"
        hw = host_cpu_info()
        threads = hw["threads_used"]
        box = {}

        def run():
            box["ref"], secs = f(*args, threads=threads, n=sample)
            return secs

        rate, passes = median_rate(run, sample)
        ref = box["ref"]
        n1 = max(1, sample // 16)
        rate1, _ = median_rate(lambda: f(*args, threads=1, n=n1)[1], n1, passes=1)
        v = np.frombuffer(self.ts.verdicts(), np.uint8)[:sample]
        mism = int((ref != v).sum())
        return dict(value=rate, unit="verifies/s", cores=threads, kind="reference",
                    sample=f"first {sample} {self.kind.upper()} tuples of rank 0, {what}, "
                           f"dynamically chunked std::thread pool x{threads}, median of "
                           f"{CPU_PASSES} passes after 1 warm-up; reference accepted "
                           f"{int(ref.sum())}/{sample}; GPU verdict mismatches on the sample: "
                           f"{mism}",
                    passes=passes, single_core_value=rate1, host=hw, gpu_verdict_mismatches=mism)

    def config(self, world):
        if self.kind == "c4":
            w = ("C4: ECDSA (pub, msg32, DER sig) tuples, 10% adversarial over 18 classes, "
                 "CPubKey::Verify semantics (BASELINE.json configs[3]; node batch = 8 x per-GPU)")
        else:
            w = ("C5: BIP340 Schnorr rows, GPU-signed + the 15 BIP340 vectors tiled "
                 "(BASELINE.json configs[4])")
        return {"workload": w, "tuples_per_gpu": self.n, "global_tuples": self.n * world,
                "parallelism": f"shard x{world} (independent tuples, no collective)"}

    @property
    def data(self):
        return f"synthetic (deterministic {self.kind.upper()} tuples, GPU-generated keys/signatures)"


class C5T:
    """BIP341 key-path Taproot spends through bcc_taproot_verify_batch:
    GenericTransactionSignatureChecker::CheckSchnorrSignature per check (interpreter.cpp:1678-1704),
    i.e. SignatureHashSchnorr over the tx + its spent outputs and the BIP340 verification, end to
    end from host buffers (host SigMsg building, H2D, GPU aux / TapSighash / Schnorr kernels)."""
    unit = "checks/s"
    data = ("synthetic (1-in/1-out key-path Taproot spends, GPU-generated keys and BIP340 "
            "signatures over the engine's own BIP341 sighashes, 5% of signatures corrupted)")

    def __init__(self, B, n, seed, dev, first=0, total=None):
        import ctypes
        import hashlib
        import numpy as np
        self.B, self.n, self.units, self.dev = B, n, n, dev
        self.mads = MADS_PER_SCHNORR
        self.kernel = "taproot end to end (host SigMsg + GPU tapsighash + schnorr prep/ladder/parity)"
        rng = np.random.default_rng(seed + first)
        d = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        d[:, 0] &= 0x7F  # < n, != 0 (w.p. 1 - 2^-120)
        d[:, 31] |= 1
        BL = B.blib()
        u8 = lambda a: a.ctypes.data_as(ctypes.c_char_p)  # noqa: E731
        sig = np.zeros((n, 64), np.uint8)
        xo = np.zeros((n, 32), np.uint8)
        ok = np.zeros(n, np.uint8)
        k = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        k[:, 0] &= 0x7F
        k[:, 31] |= 1
        m = np.zeros((n, 32), np.uint8)
        assert BL.mi_gen_schnorr_sign(u8(d), u8(m), u8(k), n, u8(sig), u8(xo), u8(ok), dev) == 0
        # tx: v2 | marker/flag | 1 input | 1 P2TR output | witness [sig64] | locktime (162 bytes)
        L = 162
        tx = np.zeros((n, L), np.uint8)
        tx[:, 0] = 2
        tx[:, 5] = 1
        tx[:, 6] = 1
        tx[:, 7:39] = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)   # prevout txid
        tx[:, 39] = rng.integers(0, 4, size=n, dtype=np.uint8)             # vout
        tx[:, 44:48] = 0xFF                                                 # nSequence
        tx[:, 48] = 1
        tx[:, 49:57] = rng.integers(0, 256, size=(n, 8), dtype=np.uint8)
        tx[:, 56] &= 0x03
        tx[:, 57] = 34
        tx[:, 58] = 0x51
        tx[:, 59] = 0x20
        tx[:, 60:92] = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
        tx[:, 92] = 1
        tx[:, 93] = 64
        tx[:, 94:158] = 0x5A
        spent = np.zeros((n, 44), np.uint8)
        spent[:, 0] = 1
        spent[:, 1:9] = rng.integers(0, 256, size=(n, 8), dtype=np.uint8)
        spent[:, 8] &= 0x03
        spent[:, 9] = 34
        spent[:, 10] = 0x51
        spent[:, 11] = 0x20
        spent[:, 12:44] = xo
        self.tx, self.spent, self.xo = tx, spent, xo
        self.sig = np.zeros((n, 64), np.uint8)
        self.leaf = np.zeros(32, np.uint8)
        T = B.TaprootCheck
        arr = (T * n)()
        base_tx, base_sp = tx.ctypes.data, spent.ctypes.data
        base_sig, base_pk = self.sig.ctypes.data, xo.ctypes.data
        vp = ctypes.c_void_p
        # fill the struct array through a numpy view (n ctypes assignments would take seconds)
        view = np.ctypeslib.as_array(ctypes.cast(arr, ctypes.POINTER(ctypes.c_uint8)),
                                     shape=(n * ctypes.sizeof(T),)).view(np.uint8)
        rec = np.zeros(1, dtype=np.dtype({"names": [f for f, _ in T._fields_],
                                          "formats": ["u8", "u4", "u8", "u4", "u4", "u8", "u4",
                                                      "u8", "i4", "u8", "u4", "u8", "u4"],
                                          "offsets": [getattr(T, f).offset for f, _ in T._fields_],
                                          "itemsize": ctypes.sizeof(T)}))
        recs = view.view(rec.dtype)
        idx = np.arange(n, dtype=np.uint64)
        recs["tx"] = base_tx + idx * L
        recs["tx_len"] = L
        recs["spent_outputs"] = base_sp + idx * 44
        recs["spent_outputs_len"] = 44
        recs["n_in"] = 0
        recs["sig"] = base_sig + idx * 64
        recs["sig_len"] = 64
        recs["pubkey32"] = base_pk + idx * 32
        recs["sigversion"] = 0
        recs["annex"] = 0
        recs["annex_len"] = 0
        recs["tapleaf_hash32"] = self.leaf.ctypes.data
        recs["codeseparator_pos"] = 0xFFFFFFFF
        self.arr = arr
        self.ret = np.zeros(n, np.int32)
        self.err = np.zeros(n, np.int32)
        Lb = B.lib()
        self.L = Lb
        hs = np.zeros((n, 32), np.uint8)
        assert Lb.bcc_taproot_verify_batch(arr, n, self._p(self.ret), self._p(self.err),
                                           hs.ctypes.data, dev) == 0
        assert BL.mi_gen_schnorr_sign(u8(d), u8(hs), u8(k), n, u8(self.sig), u8(xo), u8(ok),
                                      dev) == 0
        bad = rng.random(n) < 0.05
        self.sig[bad, rng.integers(0, 64)] ^= 0x10
        self.expect = int((~bad).sum())
        self.hs = hs
        del hashlib

    @staticmethod
    def _p(a):
        import ctypes
        return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))

    def step(self, sp):
        rc = self.L.bcc_taproot_verify_batch(self.arr, self.n, self._p(self.ret),
                                             self._p(self.err), None, self.dev)
        assert rc == 0

    def valid(self):
        self.step(None)
        return int((self.ret == 1).sum())

    def item_verdicts(self):
        return bytes((self.ret == 1).astype("uint8"))

    def kernel_times(self, stream, reps):
        t0 = time.perf_counter()
        for _ in range(reps):
            self.step(None)
        return 0.0, (time.perf_counter() - t0) / reps * 1e3

    shape = property(lambda self: {"tuples": self.n})

    def extra(self, sighash_ms):
        return {"expected_valid": self.expect,
                "note": "value = checks/s of bcc_taproot_verify_batch end to end from host buffers; "
                        "roofline = the BIP340 work unit over that end-to-end time (a lower bound "
                        "for the kernels)"}

    def cpu(self, sample):
        import ctypes
        import numpy as np
        R = _reference()
        if R is None:
            return None
        sample = min(sample, self.n)
        R.L.ref_bulk_taproot.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]
        R.L.ref_bulk_taproot.restype = ctypes.c_double
        hw = host_cpu_info()
        threads = hw["threads_used"]
        ret = np.zeros(sample, np.int32)
        err = np.zeros(sample, np.int32)
        base = ctypes.addressof(self.arr)
        rate, passes = median_rate(lambda: R.L.ref_bulk_taproot(
            threads, sample, base, ret.ctypes.data, err.ctypes.data), sample)
        n1 = max(1, sample // 16)
        rate1, _ = median_rate(lambda: R.L.ref_bulk_taproot(
            1, n1, base, ret.ctypes.data, err.ctypes.data), n1, passes=1)
        R.L.ref_bulk_taproot(threads, sample, base, ret.ctypes.data, err.ctypes.data)
        mism = int(((ret == 1) != (self.ret[:sample] == 1)).sum() +
                   ((ret == 0) & (err != self.err[:sample])).sum())
        return dict(value=rate, unit="checks/s", cores=threads, kind="reference",
                    sample=f"first {sample} C5T checks, CheckSchnorrSignature (reference "
                           f"interpreter.cpp:1678-1704 via oracle/_ref), dynamically chunked "
                           f"std::thread pool x{threads}, median of {CPU_PASSES} passes after 1 "
                           f"warm-up; reference accepted {int((ret == 1).sum())}/{sample}; "
                           f"GPU (ret, serror) mismatches on the sample: {mism}",
                    passes=passes, single_core_value=rate1, host=hw, gpu_verdict_mismatches=mism)

    def config(self, world):
        return {"workload": "C5T: BIP341 key-path Taproot spends, SignatureHashSchnorr + BIP340 "
                            "through bcc_taproot_verify_batch end to end (SURVEY 8f rank 3)",
                "checks_per_gpu": self.n, "global_checks": self.n * world,
                "parallelism": f"shard x{world} (independent checks, no collective)"}


class SideLegs:
    """The default C2 line's end-to-end legs of two other configs, on the driver's clock
    (VERDICT r05 #4): C3 block replay through bitcoinconsensus_verify_batch (4,000 txs, every
    item against the reference, its own 16-thread reference baseline) and C4 through
    bcc_pubkey_verify_batch from host buffers (8M tuples, every verdict against the staged
    kernels' and the construction labels, a reference sample).  Built and called once right after
    staging (their pinned images, device batches and scratch allocated early, as a library caller
    sets up once: DESIGN.md §3.10, allocation order), measured after C2's timed region."""

    def __init__(self, B, dev, c4_n):
        self.B, self.dev = B, dev
        t0 = time.time()
        self.c3 = C3(B, DEFAULT_N["c3"], SEEDS["c3"], dev)
        self.c3.wl.verify_batch()
        self.c4 = TupleJob(B, c4_n, SEEDS["c4"], dev, "c4") if c4_n else None
        if self.c4:
            self.c4.ts.run()  # the staged kernels' verdicts (the leg's parity reference)
            self.c4.end_to_end(self.c4.ts.host(), reps=1)
        self.setup_s = time.time() - t0

    def c3_leg(self, calls=21, cpu=True):
        import statistics
        job = self.c3
        nv, ret = job.wl.verify_batch()
        ts, runs = [], []
        for _ in range(calls):
            t0 = time.perf_counter()
            job.wl.verify_batch()
            ts.append(time.perf_counter() - t0)
            runs.append(self.B.last_batch_stats())
        med = statistics.median(ts)
        out = dict(workload=job.config(1)["workload"], inputs=job.n, calls=calls,
                   inputs_per_s=job.n / med, ms_median=med * 1e3, ms_best=min(ts) * 1e3,
                   valid=nv,
                   batch_stats_median={k: statistics.median(r[k] for r in runs)
                                       for k in ("host_seconds", "gpu_seconds", "prepare_seconds",
                                                 "interpret_seconds", "stage_seconds", "rounds",
                                                 "tuples", "early_rows", "host_hashed")})
        self._c3_ret = ret
        if cpu:
            self.c3_cpu(out)
        return out

    def c3_cpu(self, out):
        """The C3 leg's 16-thread reference baseline over all its items, with per-item verdict
        mismatches against the GPU's (measured separately from the leg's calls)."""
        job = self.c3
        cb = cpu_baseline_script([job.wl.item(i) for i in range(job.n)],
                                 f"C3 inputs (all {job.n})", gpu_verdicts=self._c3_ret)
        if cb:
            cb.pop("host", None)
            out["cpu_baseline"] = cb
            out["gpu_vs_cpu"] = out["inputs_per_s"] / cb["value"]
            out["gpu_verdict_mismatches_all_items"] = cb["gpu_verdict_mismatches"]

    def c4_leg(self, cpu=True):
        import numpy as np
        job = self.c4
        h = job.ts.host()
        e = job.end_to_end(h, reps=3)
        v = np.frombuffer(job.ts.verdicts(), np.uint8)
        e.update(workload=job.config(1)["workload"], tuples=job.n,
                 mismatches_vs_construction=int((v != h["expect"]).sum()))
        if cpu:
            cb = job.cpu(100_000)
            if cb:
                cb.pop("host", None)
                e["cpu_baseline"] = cb
                e["gpu_vs_cpu"] = e["verifies_per_s"] / cb["value"]
        return e


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=("c2", "c3", "c4", "c5", "c5t"), default="c2")
    ap.add_argument("--n", type=int, default=None,
                    help="units per GPU: inputs (c2), transactions (c3), tuples (c4, c5)")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--cpu-sample", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the drop-in / single-call / host-buffer extras (profiling runs: "
                         "every launch is then a full-size one)")
    ap.add_argument("--sustain-s", type=float, default=3.0,
                    help="after the timed steps, keep stepping for this long (HIP-event timed, "
                         "reported as `sustained`; gives a GPU-busy sampler a multi-second window)")
    ap.add_argument("--side-c4", type=int, default=8_000_000,
                    help="C2 line only: tuples of the C4 bcc_pubkey_verify_batch leg (0: no C4 leg)")
    ap.add_argument("--no-side", action="store_true",
                    help="C2 line only: skip the C3 / C4 end-to-end legs")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per ECDSA launch from a rocprofv3 --pmc run (profiles/)")
    args = ap.parse_args()
    n = args.n or DEFAULT_N[args.config]
    seed = SEEDS[args.config] if args.seed is None else args.seed

    import torch
    import torch.distributed as dist
    import bitcoinconsensus_amd as B

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    B.set_device(dev)

    t0 = time.time()
    # one global set of world x n units from `seed`; this rank's contiguous range
    first, total = rank * n, world * n
    if args.config in ("c2", "c3"):
        job = (C2 if args.config == "c2" else C3)(B, n, seed, dev, first=first, total=total)
    elif args.config == "c5t":
        job = C5T(B, n, seed, dev, first=first, total=total)
    else:
        job = TupleJob(B, n, seed, dev, args.config, first=first, total=total)
    log(f"[rank {rank}] staged {args.config} x{n} in {time.time() - t0:.1f}s")
    probe = os.environ.get("BCC_BENCH_E2E_PROBE") and args.config == "c4"

    def e2e_probe(where):  # (diagnostics: the C4 drop-in leg at points of the run)
        if probe:
            log(f"[e2e probe] {where}: {job.end_to_end(job.ts.host())['calls_ms']}")
    e2e_probe("after staging")
    side = None
    if args.config == "c2" and os.environ.get("BCC_BENCH_DROPIN_EARLY") and not args.no_extra:
        job.wl.verify_batch()  # (diagnostics: the drop-in's host state allocated first)
    if args.config == "c2" and world == 1 and not args.no_extra and not args.no_side:
        side = SideLegs(B, dev, args.side_c4)
        log(f"[rank {rank}] side legs (C3, C4 x{args.side_c4}) set up in {side.setup_s:.1f}s")
    # (the same for the C2 drop-in leg measured neutral within the boxes' noise: not done)
    early_alloc = not os.environ.get("BCC_BENCH_NO_EARLY_ALLOC")  # (A/B of the note below)
    if args.config == "c4" and not args.no_extra and early_alloc:
        # one untimed drop-in call now, so that its pinned round images, device batches and
        # scratch are allocated beside the staged set rather than after the whole run: allocated
        # last, the same calls ran ~40 % slower on the device (profiles/r05/c4_der/
        # bench_inprocess_gap.txt; a caller's buffers are normally set up once, early)
        job.end_to_end(job.ts.host(), reps=1)
    # a dedicated (non-null) stream: every launch of a step and the HIP events that time the
    # kernels sit on it (torch's default stream is the null handle, which the engine maps to its
    # own internal stream)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream

    e2e_probe("after set_stream")
    for _ in range(args.warmup):
        job.step(sp)
    torch.cuda.synchronize()
    n_valid = job.valid()
    e2e_probe("after warmup + valid")

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(args.steps):
        job.step(sp)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - ts
    elapsed, n_valid_all = aggregate(elapsed, n_valid, world)

    # sustained window: the same step back to back for >= --sustain-s seconds on every rank
    # (outside the K timed steps; a driver-side GPU-busy sampler sees a multi-second busy run)
    sustained = None
    if args.sustain_s > 0:
        per = elapsed / max(1, args.steps)
        k = max(1, int(args.sustain_s / max(per, 1e-4)))
        barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(k):
            job.step(sp)
        torch.cuda.synchronize()
        barrier()
        sus, _ = aggregate(time.perf_counter() - t1, 0, world)
        sustained = dict(steps=k, seconds=sus, value=job.units * world * k / sus,
                         ms_per_step=sus / k * 1e3)

    # the C3 block-replay leg right after the timed region (before the 1M-input drop-in calls
    # below reshape the calling thread's host state and the pinned images)
    c3_leg = side.c3_leg(cpu=False) if side else None

    # the drop-in per rank (north star: the per-input verify_batch API at 1..8 GPUs): every rank
    # calls bitcoinconsensus_verify_batch on its own slice from host buffers at the same time,
    # barrier-bracketed, max over ranks; reported beside value (host pass + H2D included)
    per_rank = None
    if args.config == "c2" and not args.no_extra:
        job.wl.verify_batch()  # warm this rank's host / device state
        best = None
        for _ in range(2):
            barrier()
            t1 = time.perf_counter()
            job.wl.verify_batch()
            dt, _ = aggregate(time.perf_counter() - t1, 0, world)
            best = dt if best is None else min(best, dt)
        per_rank = dict(inputs_per_s=job.n * world / best, ms=best * 1e3, ranks=world,
                        inputs_per_rank=job.n, host_threads_per_rank=B.host_threads(),
                        cpu_share_per_rank=B.cpu_share(),
                        note="one bitcoinconsensus_verify_batch caller per GPU on its own slice, "
                             "all ranks at once, max wall time over ranks (best of 2)")
    # the global validity bitmap (RCCL all-gather, outside the timed loop)
    gathered = gather_verdicts(bytearray(job.item_verdicts()), world)
    bitmap = dict(units=int(len(gathered)), valid=int(gathered.sum()),
                  collective="all_gather_into_tensor (RCCL)" if world > 1 else "none (1 rank)")

    e2e_probe("after timed + sustained")
    # per-kernel timing with HIP events on the launch stream (outside the timed region)
    sighash_ms, sig_ms = job.kernel_times(stream, max(3, args.steps))
    e2e_probe("after kernel_times")
    sig_units = job.shape["tuples"] if args.config in ("c2", "c3", "c5t") else job.units

    total = job.units * world * args.steps
    value = total / elapsed
    if rank == 0:
        # peak: the v_mad_u64_u32 issue limit at the spec clock (MI355X_MICROARCH.md: 2400 MHz max;
        # a wave64 v_mad_u64_u32 occupies its SIMD 4 cycles: 16 lanes/clk/SIMD x 4 SIMDs x CUs);
        # beside it the sustained on-box rate (8 independent mads per asm block, 8 waves/SIMD,
        # >= 1 s of back-to-back ~20 ms launches) and the clock it held (s_memtime stamps)
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        peak = 2.4e9 * cus * 4 * 16
        m_rate, m_clk, m_ms = B.microbench_sustained(25, 8, 20.0, 1.0, 3)
        e2e_probe("after microbench_sustained")
        achieved = sig_units * job.mads / (sig_ms * 1e-3)
        traffic, tsrc = args.traffic, "--traffic" if args.traffic else None
        tf = os.path.join(ROOT, "profiles", "traffic.json")
        if traffic is None and os.path.exists(tf):
            tj = json.load(open(tf))
            t = tj.get(f"{args.config}@{sig_units}") or tj.get(args.config)
            if t and t.get("units") == sig_units and t.get("kernel") == job.kernel:
                traffic, tsrc = t["traffic_bytes"], t["source"]
        roof = dict(bound="int-alu", kernel=job.kernel,
                    achieved=achieved / 1e12, peak=peak / 1e12, unit="T(v_mad_u64_u32)/s",
                    frac=achieved / peak, traffic=traffic, traffic_source=tsrc,
                    peak_source=f"spec: 2.4 GHz x {cus} CUs x 4 SIMDs x 16 lanes/clk "
                                "(v_mad_u64_u32, 4 cycles per wave64)",
                    peak_measured=dict(T_per_s=m_rate / 1e12, clock_GHz=m_clk,
                                       T_per_s_at_2_4GHz=m_rate / 1e12 * 2.4 / m_clk,
                                       launch_ms=m_ms, frac_vs_measured=achieved / m_rate,
                                       source="mi_microbench_sustained(op 25: 8 v_mad_u64_u32 with "
                                              "own SGPR carries per asm block, 8 waves/SIMD)"),
                    per_launch=dict(verifies=sig_units, mads=sig_units * job.mads, avg_ms=sig_ms,
                                    verifies_per_s=sig_units / (sig_ms * 1e-3)))
        cm = newest_cost_model()
        if args.config == "c2" and os.path.exists(cm):
            # why frac stops where it does (committed PMC passes + microbenchmark): the ladder is
            # VALU-issue-bound; its cycles split by instruction class at the measured issue costs
            d = json.load(open(cm))
            kname = next((n for n in ("twist_keyq_kernel", "twist_ladder_q_kernel",
                                    "twist_ladder_kernel<false>")
                          if "bench:" + n in d["kernels"]), None)
            k = d["kernels"].get("bench:" + kname) if kname else None
            if k:
                roof["cost_model"] = dict(
                    kernel=kname, cycle_share=k["cycle_share"],
                    salu_per_verify=k.get("salu_per_wave"),
                    valu_per_verify=k["valu_per_wave"],
                    issue_cost_cycles=d["issue_cost_cycles_per_wave_instr"],
                    predicted_over_measured_cycles=k["predicted_over_measured"],
                    source=os.path.relpath(cm, ROOT) + " (tools/isa/cost_model.py)")
        cpu = None
        if world == 1 and not args.no_cpu:
            default_sample = {"c2": 200_000, "c3": 100_000, "c4": 400_000, "c5": 400_000,
                              "c5t": 200_000}
            cpu = job.cpu(args.cpu_sample or default_sample[args.config])
        out = {
            "metric": METRIC, "value": value, "unit": job.unit, "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": job.data,
            "config": job.config(world),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        e2e_probe("before extra")
        if not args.no_extra:
            out.update(job.extra(sighash_ms))
        if sustained:
            out["sustained"] = sustained
        if per_rank:
            out["drop_in_per_rank"] = per_rank
        if side:
            if not args.no_cpu:
                side.c3_cpu(c3_leg)
            out["c3_block_replay"] = c3_leg
            if side.c4:
                out["c4_pubkey_verify_batch"] = side.c4_leg(cpu=not args.no_cpu)
        out["source_hash"] = B.source_hash()
        out["verdicts_valid"] = n_valid_all
        out["validity_bitmap"] = bitmap
        out["verdicts_total"] = job.units * world
        if cpu:
            out["gpu_vs_cpu"] = value / cpu["value"]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
