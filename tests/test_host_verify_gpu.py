"""GPU box: the library's host verification path (csrc/host/host_verify.cpp inside librbc_amd.so:
device-failure fallback and small rounds) gives exactly the GPU kernels' and the reference's
verdicts.

* bcc_host_verify_tuples over 20,000 tuples of the C4 set (every adversarial class) against the
  GPU verdicts of the same staged set and the reference's CPubKey::Verify (pubkey.cpp:191-207);
* bcc_set_host_small_round: the crate vectors through verify() and the script-level goldens
  through bitcoinconsensus_verify_batch with every round on the host, against the reference's
  (ret, err) (bitcoinconsensus.cpp:79-102)."""
import gzip
import json
import os

import numpy as np
import pytest

from fixtures import load_json, pub_to_tuple
from oracle_ctypes import Oracle, Reference, reference_available

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_host_verify_tuples_match_gpu_and_reference():
    import bitcoinconsensus_amd as B
    ts = B.TupleSet(20_000, kind="c4", seed=0x5EED0004)
    ts.run()
    gpu = np.frombuffer(ts.verdicts(), np.uint8)
    h = ts.host()
    ref, _ = Reference().pubkey_verify_blob(h["pub_blob"], h["pub_off"], h["msg32"],
                                            h["sig_blob"], h["sig_off"], threads=16)
    O = Oracle()
    pub, r32, s32 = bytearray(), bytearray(), bytearray()
    po, so = h["pub_off"], h["sig_off"]
    for i in range(ts.n):
        tag, x, y = pub_to_tuple(bytes(h["pub_blob"][po[i]:po[i + 1]]))
        ok, r, s = O.der_parse_lax(bytes(h["sig_blob"][so[i]:so[i + 1]]))
        pub += bytes([tag]) + x + y
        r32 += r if ok else bytes(32)
        s32 += s if ok else bytes(32)
    host = np.frombuffer(B.host_verify_tuples(bytes(pub), bytes(h["msg32"]), bytes(r32),
                                              bytes(s32), threads=16), np.uint8)
    assert (host == gpu).all(), np.nonzero(host != gpu)[0][:20]
    assert (host == np.asarray(ref, np.uint8)).all()
    assert len(set(h["cls"].tolist())) == len(B.TupleSet.C4_CLASSES)
    ts.free()


def test_small_rounds_on_host_match_reference():
    import bitcoinconsensus_amd as B
    cases = json.load(gzip.open(os.path.join(GOLDEN, "script_cases.json.gz"), "rt"))
    B.set_host_small_round(1 << 30)
    try:
        for v in load_json("crate_vectors.json"):
            got = B.verify_script_with_amount(bytes.fromhex(v["spk"]), v["amount"],
                                              bytes.fromhex(v["tx"]), v["nin"], v["flags"])
            assert got == (v["ret"], v["err"]), v["name"]
        by_flags = {}
        for c in cases:
            by_flags.setdefault(c["flags"], []).append(c)
        for flags, cs in by_flags.items():
            items = [(bytes.fromhex(c["spk"]), c["amount"], bytes.fromhex(c["tx"]), c["nin"])
                     for c in cs]
            rc, got = B.verify_batch_raw(items, flags)
            st = B.last_batch_stats()
            assert rc >= 0 and [tuple(g) for g in got] == [(c["ret"], c["err"]) for c in cs]
            assert st["host_rounds"] == st["rounds"]
    finally:
        B.set_host_small_round(0)


def test_default_small_round_threshold():
    """The library default (BCC_HOST_SMALL_ROUND_DEFAULT = 16 checks; the suite itself runs with
    0): a lone verify() is verified on the host, a batch of more checks goes to the GPU, both with
    the reference's results."""
    import bitcoinconsensus_amd as B
    vs = load_json("crate_vectors.json")
    B.set_host_small_round(B.HOST_SMALL_ROUND_DEFAULT)
    try:
        for v in vs:
            item = (bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"])
            rc, got = B.verify_batch_raw([item], v["flags"])
            st = B.last_batch_stats()
            assert [tuple(g) for g in got] == [(v["ret"], v["err"])], v["name"]
            assert st["host_rounds"] == st["rounds"]  # <= 16 checks: the host
        v = next(x for x in vs if x["name"] == "p2pkh")
        item = (bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"])
        rc, got = B.verify_batch_raw([item] * 64, v["flags"])
        st = B.last_batch_stats()
        assert [tuple(g) for g in got] == [(v["ret"], v["err"])] * 64
        assert st["rounds"] >= 1 and st["host_rounds"] == 0  # 64 checks: the GPU
    finally:
        B.set_host_small_round(0)
