"""GPU parity of the tuple level (configs C4 / C5) through the product C ABI:

* bcc_pubkey_verify_batch (N x CPubKey::Verify, pubkey.cpp:191-207) against the reference
  verdicts of the committed adversarial fixtures (tests/golden/ecdsa_tuples.npz);
* the C4 tuple set (90 % valid + 18 adversarial classes, include/bcc_amd.h bcc_tupleset_c4)
  against the reference's CPubKey::Verify on every tuple, and against the verdict by construction;
* the C5 BIP340 set (fresh GPU-signed rows + the 15 BIP340 vectors tiled) against the
  reference's secp256k1_schnorrsig_verify on every row."""
import numpy as np
import pytest

from fixtures import bip340_vectors, ecdsa_tuples
from oracle_ctypes import Reference, reference_available

pytestmark = pytest.mark.gpu
THREADS = 16


def test_pubkey_verify_batch_matches_reference_fixtures():
    import bitcoinconsensus_amd as B
    ts = ecdsa_tuples()
    v = B.pubkey_verify_batch([(t["pub"], t["hash"], t["sig"]) for t in ts])  # CPubKey level
    bad = [(t["cls"], i, v[i], t["verdict"]) for i, t in enumerate(ts) if v[i] != t["verdict"]]
    assert not bad, bad[:20]


def test_pubkey_verify_batch_empty_and_garbage():
    import bitcoinconsensus_amd as B
    assert B.pubkey_verify_batch([]) == b""
    rows = [(b"", bytes(32), b""), (b"\x02" + bytes(32), bytes(32), b"\x30\x00"),
            (b"\x04" * 65, bytes(32), b"\x30" * 70), (b"\x03" * 33, b"\xff" * 32, b"")]
    assert B.pubkey_verify_batch(rows) == bytes(4)


@pytest.fixture(scope="module")
def c4():
    import bitcoinconsensus_amd as B
    ts = B.TupleSet(300_000, kind="c4", seed=0x5EED0004)
    ts.run()
    return ts


def test_c4_classes_and_construction(c4):
    import bitcoinconsensus_amd as B
    h = c4.host()
    cls = h["cls"]
    counts = np.bincount(cls, minlength=len(B.TupleSet.C4_CLASSES))
    assert len(counts) == len(B.TupleSet.C4_CLASSES) and counts.min() > 0
    assert 0.88 < counts[0] / c4.n < 0.92
    v = np.frombuffer(c4.verdicts(), np.uint8)
    bad = np.nonzero(v != h["expect"])[0]
    assert len(bad) == 0, [(int(i), B.TupleSet.C4_CLASSES[cls[i]]) for i in bad[:20]]


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_c4_matches_reference_every_tuple(c4):
    h = c4.host()
    ref, _ = Reference().pubkey_verify_blob(h["pub_blob"], h["pub_off"], h["msg32"],
                                            h["sig_blob"], h["sig_off"], threads=THREADS)
    v = np.frombuffer(c4.verdicts(), np.uint8)
    assert np.array_equal(v, ref), np.nonzero(v != ref)[0][:20]
    assert np.array_equal(ref, h["expect"])


def test_c4_through_pubkey_verify_batch(c4):
    """The staged rows are exactly what the host front end builds: the one-shot entry point over
    the same tuples gives the same verdicts."""
    import bitcoinconsensus_amd as B
    m = 20_000
    tup = [c4.tuple(i) for i in range(m)]
    assert B.pubkey_verify_batch(tup) == c4.verdicts()[:m]


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_c5_matches_reference_every_row():
    import bitcoinconsensus_amd as B
    vec = [(t["sig"], t["msg"], t["pub"], t["verdict"]) for t in bip340_vectors()]
    ts = B.TupleSet(100_000, kind="c5", seed=0x5EED0005, vectors=vec)
    ts.run()
    v = np.frombuffer(ts.verdicts(), np.uint8)
    h = ts.host()
    ref, _ = Reference().schnorr_verify_rows(h["sig64"], h["msg32"], h["xonly32"], threads=THREADS)
    assert np.array_equal(v, ref), np.nonzero(v != ref)[0][:20]
    assert np.array_equal(v, h["expect"])
    assert (h["cls"] > 0).sum() >= len(vec) * (100_000 // 1024)


def test_c4_chunking_invariance(c4):
    """The ECDSA kernels over the same staged rows in 65,536-lane chunks (5 launch pairs) and in
    one chunk give identical verdicts."""
    import bitcoinconsensus_amd as B
    one = c4.verdicts()
    B.set_chunk_lanes(65_536)
    try:
        c4.run()
        assert c4.verdicts() == one
    finally:
        B.set_chunk_lanes(0)


def test_scratch_oom_halves_the_chunk(c4):
    """when the device cannot hold the default 16M-lane chunk scratch (other callers'
    scratch, a smaller GPU), the round runs in halved chunks on the GPU -- same verdicts, no host
    fallback (the autouse fixture checks bcc_host_fallback_rounds) and no error."""
    import bitcoinconsensus_amd as B
    B.release_thread_state()  # drop this thread's cached scratch so the next round reallocates
    B.debug_scratch_cap_lanes(100_000)  # 120,064 lanes wanted: 65,536-lane chunks fit
    try:
        h = c4.host()
        n = 120_000
        po, so = h["pub_off"][: n + 1], h["sig_off"][: n + 1]
        tuples = [(h["pub_blob"][po[i]:po[i + 1]].tobytes(), h["msg32"][32 * i:32 * i + 32].tobytes(),
                   h["sig_blob"][so[i]:so[i + 1]].tobytes()) for i in range(n)]
        v = B.pubkey_verify_batch(tuples)
    finally:
        B.debug_scratch_cap_lanes(0)
        B.release_thread_state()
    want = np.frombuffer(c4.verdicts(), np.uint8)[:n]
    got = np.frombuffer(v, np.uint8)
    assert (got == want).all(), np.nonzero(got != want)[0][:20]


def test_pipelined_tuple_round_failure():
    """bcc_pubkey_verify_batch's pipelined rounds (at least 2M tuples, tuples.cpp tuple_rounds): a
    staged round that fails (an injected transient device fault) is re-run through the
    single-round path on a fresh batch -- same verdicts, rc 0, no host fallback (the autouse
    fixture); under BCC_DEVICE_FAILURE_ERROR three faults (the staged round, its re-run and the
    retry) make the call return the error instead of a verdict."""
    import ctypes
    import bitcoinconsensus_amd as B
    n = 2_300_000
    ts = B.TupleSet(n, kind="c4", seed=0x5EED0014)
    h = ts.host()
    L = ctypes.CDLL(B.lib()._name)  # own handle: argtypes of its own
    u64p, vp = ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p
    f = L.bcc_pubkey_verify_batch
    f.argtypes = [vp, u64p, vp, vp, u64p, vp, ctypes.c_size_t, ctypes.c_int]

    def call():
        out = np.zeros(n, np.uint8)
        rc = f(h["pub_blob"].ctypes.data, h["pub_off"].ctypes.data_as(u64p), h["msg32"].ctypes.data,
               h["sig_blob"].ctypes.data, h["sig_off"].ctypes.data_as(u64p), out.ctypes.data, n, 0)
        return rc, out

    B.debug_fail_device_rounds(1)
    try:
        rc, out = call()
    finally:
        B.debug_fail_device_rounds(0)
    assert rc == 0
    bad = np.nonzero(out != h["expect"])[0]
    assert len(bad) == 0, bad[:20]
    B.set_device_failure_policy(B.DEVICE_FAILURE_ERROR)
    B.debug_fail_device_rounds(3)
    try:
        rc, _ = call()
    finally:
        B.debug_fail_device_rounds(0)
        B.set_device_failure_policy(B.DEVICE_FAILURE_HOST)
    assert rc != 0
    rc, out = call()  # and the next call is whole again
    assert rc == 0 and np.array_equal(out, h["expect"])


def test_c4_c5_bench_sizes_match_labels():
    """BASELINE.json's full sizes through the bench's own staged path (one 16M-lane chunk): every
    one of C4's 8M tuples and C5's 16M rows gets its construction label (the labels themselves are
    pinned against the reference at 300k / 100k above), and a 200k random sample of each is
    re-checked against the reference directly."""
    import bitcoinconsensus_amd as B
    rng = np.random.default_rng(44)
    vec = [(t["sig"], t["msg"], t["pub"], t["verdict"]) for t in bip340_vectors()]
    for kind, n, seed in (("c4", 8_000_000, 0x5EED0004), ("c5", 16_000_000, 0x5EED0005)):
        ts = B.TupleSet(n, kind=kind, seed=seed, vectors=vec if kind == "c5" else ())
        ts.run()
        v = np.frombuffer(ts.verdicts(), np.uint8)
        h = ts.host()
        bad = np.nonzero(v != h["expect"])[0]
        assert len(bad) == 0, (kind, bad[:20])
        if kind == "c4":  # the same 8M through the host-buffer entry point (pipelined rounds)
            import ctypes
            L = ctypes.CDLL(B.lib()._name)  # own handle: argtypes of its own
            u64p, vp = ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p
            f = L.bcc_pubkey_verify_batch
            f.argtypes = [vp, u64p, vp, vp, u64p, vp, ctypes.c_size_t, ctypes.c_int]
            out = np.zeros(n, np.uint8)
            assert f(h["pub_blob"].ctypes.data, h["pub_off"].ctypes.data_as(u64p),
                     h["msg32"].ctypes.data, h["sig_blob"].ctypes.data,
                     h["sig_off"].ctypes.data_as(u64p), out.ctypes.data, n, 0) == 0
            assert np.array_equal(out, v)
        if reference_available():
            idx = np.sort(rng.choice(n, 200_000, replace=False))
            rows = lambda a, w: np.ascontiguousarray(np.asarray(a).reshape(-1, w)[idx]).ravel()  # noqa: E731
            if kind == "c4":
                def sub_blob(blob, off):
                    parts = [bytes(blob[off[i]:off[i + 1]]) for i in idx]
                    o = np.zeros(len(parts) + 1, np.uint64)
                    o[1:] = np.cumsum([len(p) for p in parts])
                    return np.frombuffer(b"".join(parts) + b"\0", np.uint8), o
                pb, po = sub_blob(h["pub_blob"], h["pub_off"])
                sb, so = sub_blob(h["sig_blob"], h["sig_off"])
                ref, _ = Reference().pubkey_verify_blob(pb, po, rows(h["msg32"], 32), sb, so,
                                                        threads=THREADS)
            else:
                ref, _ = Reference().schnorr_verify_rows(rows(h["sig64"], 64), rows(h["msg32"], 32),
                                                         rows(h["xonly32"], 32), threads=THREADS)
            got = v[idx]
            assert np.array_equal(got, ref), (kind, np.nonzero(got != ref)[0][:20])
        del ts
