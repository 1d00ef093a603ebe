"""Verdict agreement at scale (north star: 100 % agreement on >= 10M mixed valid / invalid inputs).

    python tools/agreement.py [--c4 10000000] [--c5 4000000] [--scripts 10000000]
                              [--out profiles/r01_agreement.json]

--scripts: SCRIPT-level agreement through the drop-in batch ABI.  Chunks alternate C2 (1M P2WPKH
spends, slices of one global set) and C3 (block413567-shaped transactions, P2PKH / P2WPKH / P2SH
2-of-3); ~12 % of the items of every chunk are mutated (bcc_workload_mutate: bit flips anywhere in
the tx or in its back half, amount +-1, spent-script bit flips, truncated txs, nIn out of range).
Every item goes through bitcoinconsensus_verify_batch (host interpreter + GPU rounds) and through
the REFERENCE's bitcoinconsensus_verify_script_with_amount (oracle/_ref, 16 host threads); (ret,
err) must agree on every item.  Most chunks use VERIFY_ALL, two use P2SH|DERSIG and NONE.

C4: the adversarial ECDSA tuple set (90 % valid + 18 classes, include/bcc_amd.h bcc_tupleset_c4)
verified on the GPU, then every tuple re-verified by the REFERENCE (oracle/_ref: CPubKey::Verify of
Bitcoin Core v0.21 + libsecp256k1, 16 host threads).  C5: the BIP340 set likewise against
secp256k1_schnorrsig_verify.  Writes per-class counts and mismatches as JSON.

--host-c4 / --host-scripts: the same checks with bcc_set_host_small_round(huge), i.e. every round
verified by the engine's HOST lane code (4x64 limbs, safegcd inverses, wNAF-5 Q half,
csrc/host/host_verify.cpp) -- the path that answers every lone verify() by default (rounds of <= 16
checks).  The C4 leg goes through bcc_pubkey_verify_batch (host length filter + lax DER, then the
host lane code), the script leg through bitcoinconsensus_verify_batch.  Every record carries the
library's source_hash, so a run can be tied to the tree it tested."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-bitcoinconsensus_amd"), os.path.join(ROOT, "tests")]
import bitcoinconsensus_amd as B  # noqa: E402
from fixtures import bip340_vectors  # noqa: E402
from oracle_ctypes import Reference  # noqa: E402


def check_host_c4(n, R, threads):
    """C4 through bcc_pubkey_verify_batch with every round on the host lane code."""
    import ctypes
    t0 = time.time()
    ts = B.TupleSet(n, kind="c4")
    h = ts.host()
    t1 = time.time()
    u8p, u64p = ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)
    out = np.zeros(n, np.uint8)
    B.set_host_small_round(1 << 62)
    try:
        rc = B.lib().bcc_pubkey_verify_batch(h["pub_blob"].ctypes.data_as(u8p),
                                             h["pub_off"].ctypes.data_as(u64p),
                                             h["msg32"].ctypes.data_as(u8p),
                                             h["sig_blob"].ctypes.data_as(u8p),
                                             h["sig_off"].ctypes.data_as(u64p),
                                             out.ctypes.data_as(u8p), n, 0)
    finally:
        B.set_host_small_round(16)
    t2 = time.time()
    assert rc == 0, rc
    ref, secs = R.pubkey_verify_blob(h["pub_blob"], h["pub_off"], h["msg32"], h["sig_blob"],
                                     h["sig_off"], threads=threads)
    cls = h["cls"]
    mism = np.nonzero(out != ref)[0]
    per = {}
    for c in range(int(cls.max()) + 1):
        m = cls == c
        per[B.TupleSet.C4_CLASSES[c]] = dict(n=int(m.sum()), host_valid=int(out[m].sum()),
                                             ref_valid=int(ref[m].sum()),
                                             mismatches=int((out[m] != ref[m]).sum()))
    res = dict(config="host_c4", path="host lane code (bcc_pubkey_verify_batch, host small round)",
               n=n, host_valid=int(out.sum()), ref_valid=int(ref.sum()),
               mismatches=int(len(mism)), first_mismatches=[int(i) for i in mism[:20]],
               host_threads=B.host_threads(), generate_s=round(t1 - t0, 2),
               host_verify_s=round(t2 - t1, 2), reference_s=round(secs, 2),
               reference_threads=threads, classes=per)
    ts.free()
    print(json.dumps({k: res[k] for k in res if k != "classes"}), flush=True)
    return res


def check(kind, n, R, threads):
    t0 = time.time()
    vec = ([(t["sig"], t["msg"], t["pub"], t["verdict"]) for t in bip340_vectors()]
           if kind == "c5" else ())
    ts = B.TupleSet(n, kind=kind, vectors=vec)
    t1 = time.time()
    ts.run()
    v = np.frombuffer(ts.verdicts(), np.uint8)
    t2 = time.time()
    h = ts.host()
    if kind == "c4":
        ref, secs = R.pubkey_verify_blob(h["pub_blob"], h["pub_off"], h["msg32"], h["sig_blob"],
                                         h["sig_off"], threads=threads)
        names = B.TupleSet.C4_CLASSES
    else:
        ref, secs = R.schnorr_verify_rows(h["sig64"], h["msg32"], h["xonly32"], threads=threads)
        names = ["fresh"] + [f"bip340_{i}" for i in range(len(vec))]
    cls = h["cls"]
    mism = np.nonzero(v != ref)[0]
    per = {}
    for c in range(int(cls.max()) + 1):
        m = cls == c
        per[names[c]] = dict(n=int(m.sum()), gpu_valid=int(v[m].sum()), ref_valid=int(ref[m].sum()),
                             mismatches=int((v[m] != ref[m]).sum()))
    out = dict(config=kind, n=n, gpu_valid=int(v.sum()), ref_valid=int(ref.sum()),
               mismatches=int(len(mism)), first_mismatches=[int(i) for i in mism[:20]],
               construction_mismatches=int((ref != h["expect"]).sum()),
               generate_s=round(t1 - t0, 2), gpu_verify_s=round(t2 - t1, 3),
               reference_s=round(secs, 2), reference_threads=threads, classes=per)
    ts.free()
    print(json.dumps({k: out[k] for k in out if k != "classes"}), flush=True)
    return out


def check_scripts(total, R, threads, host=False):
    import ctypes
    L, BL = B.lib(), B.blib()
    BL.bcc_workload_mutate.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_uint64,
                                       ctypes.c_void_p]
    BL.bcc_workload_mutate.restype = ctypes.c_void_p
    BL.bcc_itemset_items.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
    BL.bcc_itemset_items.restype = ctypes.c_void_p
    BL.bcc_itemset_free.argtypes = [ctypes.c_void_p]
    L.bitcoinconsensus_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint,
                                                ctypes.c_void_p, ctypes.c_void_p]
    R.L.ref_bulk_verify_items.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_void_p,
                                          ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p]
    R.L.ref_bulk_verify_items.restype = ctypes.c_double
    shape = [tuple(t) for t in json.load(open(os.path.join(ROOT, "tests", "golden",
                                                           "block413567_shape.json")))["txs"]]
    kinds_names = ["untouched", "tx_bitflip", "tx_back_bitflip", "amount", "spk_bitflip",
                   "truncated", "nin_range"]
    done, chunk, out = 0, 0, dict(items=0, mismatches=0, valid=0, by_kind={}, by_chunk=[])
    t0 = time.time()
    while done < total:
        flags = [B.VERIFY_ALL, B.VERIFY_P2SH | B.VERIFY_DERSIG, B.VERIFY_NONE][
            0 if chunk < 8 else (chunk - 7) % 3]
        if chunk % 2 == 0:
            n = min(1_000_000, total - done)
            wl = B.Workload(n, seed=0x5EED0001, first=done)
            kind = "c2"
        else:
            ntx = 60 * len(shape)  # ~190k inputs
            wl = B.Workload(kind="block", shape=(shape * 60)[:ntx], seed=0x5EED0003 + chunk)
            kind = "c3"
        n = wl.n
        kinds = np.zeros(n, np.uint8)
        ms = BL.bcc_workload_mutate(wl.h, 0.12, 0xA9EE + chunk, kinds.ctypes.data)
        cnt = ctypes.c_size_t()
        items = BL.bcc_itemset_items(ms, ctypes.byref(cnt))
        ret = np.zeros(n, np.int32)
        err = np.zeros(n, np.int32)
        g0 = time.time()
        if host:
            B.set_host_small_round(1 << 62)
        try:
            rc = L.bitcoinconsensus_verify_batch(items, n, flags, ret.ctypes.data, err.ctypes.data)
        finally:
            B.set_host_small_round(16)
        g1 = time.time()
        st = B.last_batch_stats()
        rret = np.zeros(n, np.int32)
        rerr = np.zeros(n, np.int32)
        rs = R.L.ref_bulk_verify_items(threads, n, items, flags, rret.ctypes.data,
                                       rerr.ctypes.data)
        bad = np.nonzero((ret != rret) | (err != rerr))[0]
        for k in range(len(kinds_names)):
            m = kinds == k
            e = out["by_kind"].setdefault(kinds_names[k], dict(n=0, ref_valid=0, mismatches=0))
            e["n"] += int(m.sum())
            e["ref_valid"] += int(rret[m].sum())
            e["mismatches"] += int(((ret != rret) | (err != rerr))[m].sum())
        rec = dict(chunk=chunk, workload=kind, flags=flags, items=n, rc=int(rc),
                   host_rounds=int(st["host_rounds"]), rounds=int(st["rounds"]),
                   gpu_valid=int(ret.sum()), ref_valid=int(rret.sum()), mismatches=int(len(bad)),
                   first_mismatches=[int(i) for i in bad[:10]],
                   verify_batch_s=round(g1 - g0, 2), reference_s=round(rs, 2),
                   elapsed_s=round(time.time() - t0, 1))
        print(json.dumps(rec), flush=True)
        out["by_chunk"].append(rec)
        out["items"] += n
        out["mismatches"] += int(len(bad))
        out["valid"] += int(rret.sum())
        BL.bcc_itemset_free(ms)
        wl.free()
        done += n
        chunk += 1
    out.update(config="host_scripts" if host else "scripts", reference_threads=threads,
               mutated_rate=0.12,
               path=("every round on the host lane code (host small round)" if host else
                     "device rounds (GPU sighash + ECDSA kernels)"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4", type=int, default=10_000_000)
    ap.add_argument("--c5", type=int, default=4_000_000)
    ap.add_argument("--scripts", type=int, default=0)
    ap.add_argument("--host-c4", type=int, default=0)
    ap.add_argument("--host-scripts", type=int, default=0)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "agreement.json"))
    a = ap.parse_args()
    R = Reference()
    res = []
    if a.c4:
        res.append(check("c4", a.c4, R, a.threads))
    if a.c5:
        res.append(check("c5", a.c5, R, a.threads))
    if a.scripts:
        res.append(check_scripts(a.scripts, R, a.threads))
    if a.host_c4:
        res.append(check_host_c4(a.host_c4, R, a.threads))
    if a.host_scripts:
        res.append(check_scripts(a.host_scripts, R, a.threads, host=True))
    for r in res:
        r["source_hash"] = B.source_hash()
        r["host_fallback_rounds"] = B.host_fallback_rounds()
    json.dump(res, open(a.out, "w"), indent=1)
    assert all(r["mismatches"] == 0 for r in res), "GPU / reference verdicts differ"


if __name__ == "__main__":
    main()
