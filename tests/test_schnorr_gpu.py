"""GPU parity of the BIP340 path (config C5): the HIP kernels behind mi_schnorr_verify_tuples vs
the reference's secp256k1_schnorrsig_verify verdicts (BIP340 vectors + tests/golden/
schnorr_tuples.npz), vs the oracle on GPU-signed random rows, and a size-independent check
across several device chunks."""
import random

import numpy as np
import pytest

from fixtures import bip340_vectors, schnorr_tuples
from oracle_ctypes import Oracle

pytestmark = pytest.mark.gpu
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _verify(rows):
    import bitcoinconsensus_amd as B
    return B.schnorr_verify_tuples(b"".join(t["sig"] for t in rows),
                                   b"".join(t["msg"] for t in rows),
                                   b"".join(t["pub"] for t in rows))


def test_schnorr_kernel_bip340_vectors_and_fixtures():
    ts = bip340_vectors() + schnorr_tuples()
    v = _verify(ts)
    bad = [(t["cls"], i, v[i], t["verdict"]) for i, t in enumerate(ts) if v[i] != t["verdict"]]
    assert not bad, bad[:20]


def _gen(n, seed):
    import bitcoinconsensus_amd as B
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    d[:, 0] &= 0x7F  # < n
    d[:, 31] |= 1    # != 0
    m = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    k = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    k[:, 0] &= 0x7F
    k[:, 31] |= 1
    sig, xo, ok = B.gen_schnorr_sign(d.tobytes(), m.tobytes(), k.tobytes())
    assert all(ok)
    return (np.frombuffer(sig, np.uint8).reshape(n, 64).copy(), m,
            np.frombuffer(xo, np.uint8).reshape(n, 32).copy())


def test_schnorr_kernel_random_vs_oracle():
    import bitcoinconsensus_amd as B
    O = Oracle()
    n = 2000
    sig, msg, pk = _gen(n, 11)
    rng = random.Random(11)
    for i in range(n):
        k = rng.randrange(5)
        if k == 1:
            msg[i, rng.randrange(32)] ^= 1 << rng.randrange(8)
        elif k == 2:
            sig[i, rng.randrange(64)] ^= 1 << rng.randrange(8)
        elif k == 3:
            pk[i, rng.randrange(32)] ^= 1 << rng.randrange(8)
    v = B.schnorr_verify_tuples(sig.tobytes(), msg.tobytes(), pk.tobytes())
    exp = [O.schnorr_verify(bytes(sig[i]), bytes(msg[i]), bytes(pk[i])) for i in range(n)]
    assert list(v) == exp
    assert 0 < sum(exp) < n


def test_schnorr_kernel_multi_chunk_property():
    """600k GPU-signed rows (3 device chunks): every signature verifies, and exactly the rows
    whose message was altered afterwards do not."""
    import bitcoinconsensus_amd as B
    n = 600_000
    sig, msg, pk = _gen(n, 12)
    B.set_chunk_lanes(262_144)  # 3 launches of the kernel pair (the default chunk holds 16M)
    try:
        v = np.frombuffer(B.schnorr_verify_tuples(sig.tobytes(), msg.tobytes(), pk.tobytes()), np.uint8)
        assert v.all()
        bad = np.arange(0, n, 7)
        msg[bad, 5] ^= 0x10
        v = np.frombuffer(B.schnorr_verify_tuples(sig.tobytes(), msg.tobytes(), pk.tobytes()), np.uint8)
        want = np.ones(n, np.uint8)
        want[bad] = 0
        assert np.array_equal(v, want)
        # the same rows in one chunk give the same verdicts
        B.set_chunk_lanes(0)
        v1 = np.frombuffer(B.schnorr_verify_tuples(sig.tobytes(), msg.tobytes(), pk.tobytes()), np.uint8)
        assert np.array_equal(v1, want)
    finally:
        B.set_chunk_lanes(0)
