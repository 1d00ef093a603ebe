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


def _small_round_env():
    """The host small-round setting the suite runs under (conftest.py sets BCC_HOST_SMALL_ROUND)."""
    import os
    return int(os.environ.get("BCC_HOST_SMALL_ROUND", "16"))


def _der_int(v, pad=0, longform=0):
    """DER INTEGER of big-endian bytes v with `pad` extra leading zero bytes; longform k > 0 writes
    the length as 0x80 | k followed by k bytes (leading zero bytes included)."""
    body = b"\x00" * pad + v
    if longform:
        ln = bytes([0x80 | longform]) + len(body).to_bytes(longform, "big")
    else:
        ln = bytes([len(body)])
    return b"\x02" + ln + body


def _der_split(sig):
    """(r, s) big-endian minimal bytes of a strict DER signature."""
    assert sig[0] == 0x30
    rl = sig[3]
    r = sig[4:4 + rl]
    s = sig[6 + rl:6 + rl + sig[5 + rl]]
    return r.lstrip(b"\x00") or b"\x00", s.lstrip(b"\x00") or b"\x00"


def _der_variants(r, s, rng):
    """Lax-DER encodings of (r, s) (pubkey.cpp:28-168): the ones a lax parser accepts with the same
    (r, s), the ones it maps to (0, 0) (an integer > 32 bytes or >= n: overflow), and malformed
    ones (parse failure)."""
    n = (0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141).to_bytes(32, "big")
    seq = lambda b, hdr=None: b"\x30" + (bytes([len(b)]) if hdr is None else hdr) + b  # noqa: E731
    ri, si = _der_int(r), _der_int(s)
    out = [
        seq(ri + si),                                        # strict
        seq(_der_int(r, pad=3) + si),                        # zero-padded r (r_zeropad), lax ok
        seq(ri + _der_int(s, pad=40)),                       # s padded past 32 bytes: still s
        seq(_der_int(r, longform=2) + si),                   # long-form length of r
        seq(ri + _der_int(s, longform=3)),                   # 3 length bytes (< 4): ok
        seq(ri + _der_int(s, longform=4)),                   # 4 length bytes, zeros skipped: ok
        seq(ri + b"\x02\x84\x01\x00\x00\x20" + s),            # 4 significant length bytes: failure
        seq(_der_int(r, longform=1, pad=1) + si),
        seq(ri + si, hdr=b"\x85\x00\x00\x00\x00\x00"),       # sequence long form (skipped)
        seq(ri + si, hdr=b"\x00"),                           # sequence length ignored
        seq(ri + si, hdr=b"\x88"),                           # sequence long form past the end
        seq(ri + si) + bytes(rng.randrange(1, 9)),           # trailing bytes (lax: ignored)
        seq(_der_int(b"\x01" + r.rjust(32, b"\x00")) + si),  # 33 significant bytes: overflow
        seq(_der_int(n) + si),                               # r = n: overflow
        seq(ri + _der_int(n)),                               # s = n
        seq(_der_int(b"\x00") + si),                         # r = 0
        seq(ri + _der_int(b"")),                             # s empty
        seq(ri + si)[:rng.randrange(1, 8 + len(r))],         # truncated
        b"", b"\x30", b"\x30\x00\x02", b"\x31" + seq(ri + si)[1:],
        seq(ri + b"\x03" + si[1:]),                          # wrong tag of S
        bytes(rng.randrange(256) for _ in range(rng.randrange(1, 80))),
    ]
    return out


def _der_variant_set():
    """Lax-DER variants of valid fixture signatures and pubkeys of every header, shuffled, as
    (tuples, pub_blob, pub_off, msg, sig_blob, sig_off)."""
    import random
    rng = random.Random(0xDE5)
    base = [t for t in ecdsa_tuples() if t["verdict"] == 1 and t["sig"][:1] == b"\x30"]
    tuples = []
    for t in base[:400]:
        try:
            r, s = _der_split(t["sig"])
        except (IndexError, AssertionError):
            continue
        pub = t["pub"]
        pubs = [pub]
        if len(pub) == 65:  # hybrid headers (both parities), a truncated key
            pubs += [bytes([6]) + pub[1:], bytes([7]) + pub[1:], pub[:33]]
        else:
            pubs += [b"\x04" + pub[1:], pub + b"\x00", b""]
        for sig in _der_variants(r, s, rng):
            tuples.append((pub, t["hash"], sig))
        for p in pubs[1:]:
            tuples.append((p, t["hash"], t["sig"]))
    rng.shuffle(tuples)
    assert len(tuples) > 5000
    pb = np.frombuffer(b"".join(t[0] for t in tuples) + b"\0", np.uint8)
    po = np.zeros(len(tuples) + 1, np.uint64)
    po[1:] = np.cumsum([len(t[0]) for t in tuples])
    sb = np.frombuffer(b"".join(t[2] for t in tuples) + b"\0", np.uint8)
    so = np.zeros(len(tuples) + 1, np.uint64)
    so[1:] = np.cumsum([len(t[2]) for t in tuples])
    msg = np.frombuffer(b"".join(t[1] for t in tuples), np.uint8)
    return tuples, pb, po, msg, sb, so


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_der_on_device_matches_reference():
    """K_der (der.hip, round 5): bcc_pubkey_verify_batch parses the caller's blobs on the device.
    Lax-DER variants of valid signatures (zero padding, long-form lengths, sequence-length garbage,
    trailing bytes, >32-byte integers, r or s >= n, zero, truncation, wrong tags, random bytes),
    pubkeys of every header and wrong lengths, all against the reference's CPubKey::Verify tuple by
    tuple, through one round and through the pipelined rounds of a 2.1M-tuple call (the variants
    tiled), and equal to the host parse (a host-lane round)."""
    import bitcoinconsensus_amd as B
    tuples, pb, po, msg, sb, so = _der_variant_set()
    ref, _ = Reference().pubkey_verify_blob(pb, po, msg, sb, so, threads=THREADS)
    got = np.frombuffer(B.pubkey_verify_batch(tuples), np.uint8)
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:20]
    assert 0.2 < ref.mean() < 0.8  # both outcomes well represented
    # the host parse (every round on the host lane code) agrees
    B.set_host_small_round(1 << 30)
    try:
        host = np.frombuffer(B.pubkey_verify_batch(tuples[:3000]), np.uint8)
    finally:
        B.set_host_small_round(_small_round_env())
    assert np.array_equal(host, ref[:3000])
    # offsets out of order anywhere (a tuple past the blob, a tuple running backwards) are an
    # argument error, on the device and on the host lane code alike: no verdict may depend on how
    # the call is cut into rounds (each round checks against its own uploaded span)
    import ctypes
    L = ctypes.CDLL(B.lib()._name)
    u64p, vp = ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p
    f = L.bcc_pubkey_verify_batch
    f.argtypes = [vp, u64p, vp, vp, u64p, vp, ctypes.c_size_t, ctypes.c_int]
    m = 4000
    for small in (_small_round_env(), 1 << 30):
        B.set_host_small_round(small)
        try:
            for which in ("past", "backwards"):
                po2, so2 = po[:m + 1].copy(), so[:m + 1].copy()
                if which == "past":
                    po2[100] = 1 << 40
                else:
                    so2[200] = so2[199] - 1
                out = np.zeros(m, np.uint8)
                assert f(pb.ctypes.data, po2.ctypes.data_as(u64p), msg.ctypes.data, sb.ctypes.data,
                         so2.ctypes.data_as(u64p), out.ctypes.data, m, 0) == -1, (small, which)
        finally:
            B.set_host_small_round(_small_round_env())
    # the pipelined rounds (>= 512k tuples: rounds staged while the previous one runs)
    reps = (2_100_000 + len(tuples) - 1) // len(tuples)
    big = tuples * reps
    got_big = np.frombuffer(B.pubkey_verify_batch(big), np.uint8)
    assert np.array_equal(got_big, np.tile(ref, reps))


_SMALL_ROUNDS_CHILD = """
import ctypes, sys
import numpy as np
sys.path.insert(0, sys.argv[2])
import bitcoinconsensus_amd as B
d = np.load(sys.argv[1])
pb, po, msg, sb, so = (np.ascontiguousarray(d[k]) for k in ("pb", "po", "msg", "sb", "so"))
n = len(po) - 1
L = ctypes.CDLL(B.lib()._name)
u64p, vp = ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p
f = L.bcc_pubkey_verify_batch
f.argtypes = [vp, u64p, vp, vp, u64p, vp, ctypes.c_size_t, ctypes.c_int]

def call(po, so):
    out = np.zeros(n, np.uint8)
    rc = f(pb.ctypes.data, po.ctypes.data_as(u64p), msg.ctypes.data, sb.ctypes.data,
           so.ctypes.data_as(u64p), out.ctypes.data, n, 0)
    return rc, out

res = {}
rc, res["plain"] = call(po, so)
assert rc == 0, rc
for k in (1, 2):  # a staged round fails: the round's rows re-parsed on the host, re-run
    B.debug_fail_device_rounds(k)
    try:
        rc, res["fault%d" % k] = call(po, so)
    finally:
        B.debug_fail_device_rounds(0)
    assert rc == 0, rc
po2 = po.copy()
po2[n // 2] = po2[n // 2 + 1] + 1  # out of order in a middle round: an argument error
assert call(po2, so)[0] == -1
assert B.host_fallback_rounds() == 0
np.savez(sys.argv[3], **res)
print("ok")
"""


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_der_variants_through_small_pipelined_rounds(tmp_path):
    """The lax-DER / pubkey variants through bcc_pubkey_verify_batch's pipelined rounds
    (tuple_rounds) with the round sizes shrunk (BCC_TUPLE_FIRST=512, BCC_TUPLE_ROUND=1024, read
    once at load: a child process), so a ~6k-tuple call runs ~7 rounds on the three-slot
    K_der staging, each round checking its own offset span: every verdict equals the reference's,
    also when a staged round fails (one and two injected faults: the round's host re-parse and the
    single-round path), and offsets out of order in a middle round are an argument error."""
    import os
    import subprocess
    import sys
    tuples, pb, po, msg, sb, so = _der_variant_set()
    ref, _ = Reference().pubkey_verify_blob(pb, po, msg, sb, so, threads=THREADS)
    inp, outp = tmp_path / "in.npz", tmp_path / "out.npz"
    np.savez(inp, pb=pb, po=po, msg=msg, sb=sb, so=so)
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "rust-bitcoinconsensus_amd")
    env = dict(os.environ, BCC_TUPLE_FIRST="512", BCC_TUPLE_ROUND="1024")
    p = subprocess.run([sys.executable, "-c", _SMALL_ROUNDS_CHILD, str(inp), pkg, str(outp)],
                       capture_output=True, text=True, timeout=100, env=env)
    assert p.returncode == 0 and "ok" in p.stdout, (p.returncode, p.stdout, p.stderr[-3000:])
    got = np.load(outp)
    for k in ("plain", "fault1", "fault2"):
        assert np.array_equal(got[k], ref), (k, np.nonzero(got[k] != ref)[0][:20])
