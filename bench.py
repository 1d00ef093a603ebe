"""bench.py — ECDSA verifies/s of the MI355X signature hot path (BASELINE.json metric, config C2).

    python bench.py [--gpus N --steps K --warmup W --n INPUTS_PER_GPU]
    (N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
             --master-port P bench.py --gpus N ...)

Workload (BASELINE.json configs[1]): n synthetic P2WPKH spends per GPU (default
1,000,000), inputs resident in HBM (staged by the engine's own first-round interpreter pass).
One step = one pass of the hot path over the batch: BIP143 sighash kernels (aux hashes, patch,
preimage SHA-256d) + the ECDSA verify kernel (pubkey decompression, s^-1, GLV, Strauss ladder,
x-check).  value = verifies of all ranks / max-over-ranks wall time of K steps.  Multi-GPU is
weak scaling: every rank verifies its own shard (seed + rank), no collective in the timed loop.

Also reported:
  roofline      the ECDSA kernel against the measured v_mad_u64_u32 issue rate (int-ALU bound:
                MFMA is deliberately unused; SURVEY.md §8d W = 2,257 modmuls = 144,448 32x32->64
                partial products per verify), kernel time from HIP events on the launch stream
  cpu_baseline  the REFERENCE (oracle/_ref: Bitcoin Core v0.21 libbitcoinconsensus built from
                /root/reference) bitcoinconsensus_verify_script_with_amount on a bounded sample of
                the same inputs, std::thread pool over the host cores (rank 0, N = 1 only)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))

MADS_PER_VERIFY = 144448          # 2,257 modmuls x 64 (32x32->64) products
METRIC = "ECDSA verifies/sec (node) at 1/2/4/8 MI355X; % of int-ALU roofline"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(wl, sample, threads):
    """Reference libbitcoinconsensus on `sample` items of the workload (checker-side code)."""
    import ctypes
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_consensus.so")
    if not os.path.exists(ref):
        return None
    L = ctypes.CDLL(ref)
    L.ref_bench_verify_script.restype = ctypes.c_double
    spks, txs, amts, nins = [], [], [], []
    for i in range(sample):
        s, a, t, k = wl.item(i)
        spks.append(s)
        txs.append(t)
        amts.append(a)
        nins.append(k)

    def blob(parts):
        off = [0]
        for p in parts:
            off.append(off[-1] + len(p))
        return b"".join(parts), (ctypes.c_long * len(off))(*off)

    sb, so = blob(spks)
    tb, to = blob(txs)
    am = (ctypes.c_int64 * sample)(*amts)
    nin = (ctypes.c_uint * sample)(*nins)
    ret = (ctypes.c_int * sample)()
    args = (ctypes.c_long(sample), sb, so, tb, to, am, nin, ctypes.c_uint(0xE15), ret)
    L.ref_bench_verify_script(ctypes.c_int(threads), ctypes.c_long(min(sample, 2000)), *args[1:])  # warm
    secs = L.ref_bench_verify_script(ctypes.c_int(threads), *args)
    ok = sum(ret[i] for i in range(sample))
    n1 = max(1, sample // 16)
    secs1 = L.ref_bench_verify_script(ctypes.c_int(1), ctypes.c_long(n1), *args[1:])
    return dict(value=sample / secs, unit="verifies/s", cores=threads, kind="reference",
                sample=f"{sample} C2 inputs (first {sample} of rank 0's workload), "
                       f"bitcoinconsensus_verify_script_with_amount flags=0xE15, "
                       f"std::thread pool x{threads}; reference accepted {ok}/{sample}",
                single_core_value=n1 / secs1, cpu_seconds=secs * threads)


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1_000_000, help="P2WPKH inputs per GPU")
    ap.add_argument("--seed", type=int, default=0x5EED0001)
    ap.add_argument("--cpu-sample", type=int, default=200_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", type=float, default=None,
                    help="HBM bytes per ECDSA launch from a rocprofv3 --pmc run (profiles/)")
    args = ap.parse_args()

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

    t0 = time.time()
    wl = B.Workload(args.n, seed=args.seed + rank, device=dev)
    shape = wl.shape()
    log(f"[rank {rank}] staged {args.n} P2WPKH inputs in {time.time() - t0:.1f}s: {shape}")
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    for _ in range(args.warmup):
        wl.run(sp)
    torch.cuda.synchronize()
    v = wl.verdicts()
    n_valid = sum(v)
    if n_valid != len(v):
        log(f"[rank {rank}] WARNING: {len(v) - n_valid} of {len(v)} verdicts invalid")

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(args.steps):
        wl.run(sp)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - ts
    elapsed, n_valid_all = aggregate(elapsed, n_valid, world)

    # per-kernel timing with HIP events on the launch stream (outside the timed region)
    reps = max(3, args.steps)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record(stream)
    for _ in range(reps):
        wl.run_sighash(sp)
    e[1].record(stream)
    for _ in range(reps):
        wl.run_ecdsa(sp)
    e[2].record(stream)
    torch.cuda.synchronize()
    sighash_ms = e[0].elapsed_time(e[1]) / reps
    ecdsa_ms = e[1].elapsed_time(e[2]) / reps

    total = shape["tuples"] * world * args.steps
    value = total / elapsed
    if rank == 0:
        peak = B.microbench(0, 4096)  # v_mad_u64_u32 lane-ops/s, measured on this GPU
        achieved = shape["tuples"] * MADS_PER_VERIFY / (ecdsa_ms * 1e-3)
        roof = dict(bound="int-alu", kernel="ecdsa_verify_kernel",
                    achieved=achieved / 1e12, peak=peak / 1e12, unit="T(v_mad_u64_u32)/s",
                    frac=achieved / peak, traffic=args.traffic,
                    per_launch=dict(verifies=shape["tuples"], mads=shape["tuples"] * MADS_PER_VERIFY,
                                    avg_ms=ecdsa_ms))
        sh_bytes = 64 * (shape["sighash_blocks"] + shape["aux_blocks"]) + 32 * (shape["preimages"] + shape["aux_messages"])
        sighash = dict(kernels="sha256d aux + patch + sha256d preimage", avg_ms=sighash_ms,
                       algorithmic_bytes=sh_bytes, achieved_GBps=sh_bytes / (sighash_ms * 1e-3) / 1e9,
                       peak_GBps=8000.0)
        cpu = None
        if world == 1 and not args.no_cpu:
            threads = min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(wl, min(args.cpu_sample, args.n), threads)
        out = {
            "metric": METRIC, "value": value, "unit": "verifies/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (deterministic P2WPKH spends, GPU-generated keys/signatures)",
            "config": {"workload": "C2: synthetic P2WPKH inputs, BIP143 sighash + ECDSA verify "
                                   "(BASELINE.json configs[1])",
                       "inputs_per_gpu": args.n, "global_inputs": args.n * world,
                       "parallelism": f"shard x{world} (independent tuples, no collective)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "sighash_stage": sighash,
            "verdicts_valid": n_valid_all, "verdicts_total": shape["tuples"] * world,
        }
        if cpu:
            out["gpu_vs_cpu"] = value / cpu["value"]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
