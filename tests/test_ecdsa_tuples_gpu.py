"""GPU parity: the HIP ECDSA kernel (inner tuple C-ABI mi_ecdsa_verify_tuples) vs the reference
verdicts in tests/golden/ecdsa_tuples.npz and vs the oracle on seeded random tuples."""
import random

import numpy as np
import pytest

from fixtures import ecdsa_tuples, pub_to_tuple
from oracle_ctypes import Oracle

pytestmark = pytest.mark.gpu
O = Oracle()


def _pack(tuples):
    pub65, msg, r32, s32 = bytearray(), bytearray(), bytearray(), bytearray()
    for t in tuples:
        tag, x, y = pub_to_tuple(t["pub"])
        ok, r, s = O.der_parse_lax(t["sig"])  # checker-side parse for the raw tuple ABI
        if not ok:
            r = s = bytes(32)
        pub65 += bytes([tag]) + x + y
        msg += t["hash"]
        r32 += r
        s32 += s
    return bytes(pub65), bytes(msg), bytes(r32), bytes(s32)


def test_ecdsa_kernel_matches_reference_fixtures():
    import bitcoinconsensus_amd as B
    ts = ecdsa_tuples()
    v = B.ecdsa_verify_tuples(*_pack(ts))
    bad = [(t["cls"], i, v[i], t["verdict"]) for i, t in enumerate(ts) if v[i] != t["verdict"]]
    assert not bad, bad[:20]


def test_ecdsa_kernel_random_vs_oracle():
    import bitcoinconsensus_amd as B
    rng = random.Random(1234)
    ts = ecdsa_tuples()
    valid = [t for t in ts if t["verdict"] == 1]
    sample = []
    for i in range(3000):
        t = dict(rng.choice(valid))
        k = rng.randrange(4)
        if k == 1:
            h = bytearray(t["hash"]); h[rng.randrange(32)] ^= 1 << rng.randrange(8); t["hash"] = bytes(h)
        elif k == 2:
            s = bytearray(t["sig"]); j = rng.randrange(8, len(s)); s[j] ^= 1 << rng.randrange(8); t["sig"] = bytes(s)
        sample.append(t)
    v = B.ecdsa_verify_tuples(*_pack(sample))
    exp = [O.pubkey_verify(t["pub"], t["hash"], t["sig"]) for t in sample]
    assert list(v) == exp


def test_ecdsa_tuples_concurrent_threads():
    """mi_ecdsa_verify_tuples from 6 threads at once (each with its own scratch + stream) returns
    the reference fixture verdicts in every thread."""
    import threading
    import bitcoinconsensus_amd as B
    ts = ecdsa_tuples()
    packed = _pack(ts)
    exp = bytes(t["verdict"] for t in ts)
    out = []

    def work():
        for _ in range(3):
            out.append(B.ecdsa_verify_tuples(*packed) == exp)

    th = [threading.Thread(target=work) for _ in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert len(out) == 18 and all(out)
