"""GPU parity of the drop-in C ABI (librbc_amd.so: host interpreter + HIP sighash + HIP ECDSA)
against the reference's verdicts on the reference's own test data and the crate vectors."""
import gzip
import json
import os

import pytest

from fixtures import load_json

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def cases():
    return json.load(gzip.open(os.path.join(HERE, "golden", "script_cases.json.gz"), "rt"))


def test_crate_vectors_rust_api():
    import bitcoinconsensus_amd as B
    vs = {v["name"]: v for v in load_json("crate_vectors.json")}
    for name in ("p2pkh", "p2sh_p2wpkh", "p2wsh_2of3"):
        v = vs[name]
        B.verify(bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"])
    for name in ("p2pkh_wrong_script", "p2sh_p2wpkh_wrong_amount", "p2wsh_wrong_program"):
        v = vs[name]
        with pytest.raises(B.ConsensusError) as ei:
            B.verify(bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"])
        assert ei.value.error == B.Error.ERR_SCRIPT
    with pytest.raises(B.ConsensusError) as ei:  # invalid_flags_test (src/lib.rs:276)
        B.verify_with_flags(b"", 0, b"", 0, B.VERIFY_ALL + 1)
    assert ei.value.error == B.Error.ERR_INVALID_FLAGS
    assert B.version() == 1


def test_script_cases_single_calls():
    import bitcoinconsensus_amd as B
    bad = []
    for c in cases():
        got = B.verify_script_with_amount(bytes.fromhex(c["spk"]), c["amount"], bytes.fromhex(c["tx"]),
                                          c["nin"], c["flags"])
        if got != (c["ret"], c["err"]):
            bad.append((c["src"], c["flags"], got, (c["ret"], c["err"])))
    assert not bad, bad[:10]


def test_script_cases_batch():
    import bitcoinconsensus_amd as B
    allc = cases()
    for flags in sorted({c["flags"] for c in allc}):
        cs = [c for c in allc if c["flags"] == flags]
        res = B.verify_batch([(bytes.fromhex(c["spk"]), c["amount"], bytes.fromhex(c["tx"]), c["nin"])
                              for c in cs], flags)
        assert [(r, int(e)) for r, e in res] == [(c["ret"], c["err"]) for c in cs]
    st = B.last_batch_stats()
    assert st["items"] > 0


def test_concurrent_callers():
    """The reference ABI is reentrant: threads calling the drop-in concurrently (ctypes
    drops the GIL for the call) must get exactly the single-threaded verdicts; each thread owns its
    device arena, scratch and stream."""
    import threading
    import bitcoinconsensus_amd as B
    allc = [c for c in cases() if c["flags"] == 0xE15][:600]
    exp = [(c["ret"], c["err"]) for c in allc]
    args = [(bytes.fromhex(c["spk"]), c["amount"], bytes.fromhex(c["tx"]), c["nin"]) for c in allc]
    errors = []

    def single(k):
        for i in range(k, len(allc), 4):
            got = B.verify_script_with_amount(args[i][0], args[i][1], args[i][2], args[i][3], 0xE15)
            if got != exp[i]:
                errors.append(("single", i, got, exp[i]))

    def batch(k):
        for _ in range(3):
            res = B.verify_batch(args[k::2], 0xE15)
            if [(r, int(e)) for r, e in res] != exp[k::2]:
                errors.append(("batch", k))

    th = [threading.Thread(target=single, args=(k,)) for k in range(4)]
    th += [threading.Thread(target=batch, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
