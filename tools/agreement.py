"""Verdict agreement at scale (north star: 100 % agreement on >= 10M mixed valid / invalid inputs).

    python tools/agreement.py [--c4 10000000] [--c5 4000000] [--out profiles/r01_agreement.json]

C4: the adversarial ECDSA tuple set (90 % valid + 18 classes, include/bcc_amd.h bcc_tupleset_c4)
verified on the GPU, then every tuple re-verified by the REFERENCE (oracle/_ref: CPubKey::Verify of
Bitcoin Core v0.21 + libsecp256k1, 16 host threads).  C5: the BIP340 set likewise against
secp256k1_schnorrsig_verify.  Writes per-class counts and mismatches as JSON."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4", type=int, default=10_000_000)
    ap.add_argument("--c5", type=int, default=4_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "agreement.json"))
    a = ap.parse_args()
    R = Reference()
    res = []
    if a.c4:
        res.append(check("c4", a.c4, R, a.threads))
    if a.c5:
        res.append(check("c5", a.c5, R, a.threads))
    json.dump(res, open(a.out, "w"), indent=1)
    assert all(r["mismatches"] == 0 for r in res), "GPU / reference verdicts differ"


if __name__ == "__main__":
    main()
