"""CPU: the kernel's per-lane arithmetic (csrc/ecdsa_lane.h, compiled for the host by
tests/native/lane_host.cpp -- test-only, never part of the product) against the reference
fixtures. Lets the exact lane code be checked without a GPU."""
import ctypes
import os
import random
import subprocess

import pytest

from fixtures import bip340_vectors, ecdsa_tuples, pub_to_tuple, schnorr_tuples
from oracle_ctypes import Oracle, Reference, reference_available

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "_build", "lane_host.so")


@pytest.fixture(scope="module")
def lane():
    src = os.path.join(HERE, "native", "lane_host.cpp")
    deps = [src] + [os.path.join(HERE, "..", "rust-bitcoinconsensus_amd", "csrc", f)
                    for f in ("ecdsa_lane.h", "ecdsa_twist.h", "secp256k1_device.h", "modinv_host.h",
                              "modinv_device.h", "sha256_device.h")]
    if not os.path.exists(SO) or any(os.path.getmtime(d) > os.path.getmtime(SO) for d in deps):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO, src])
    return ctypes.CDLL(SO)


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_lane_schnorr_twist_matches_reference_fixtures(lane):
    """BIP340 on the square-root-free path: the 15 BIP340 vectors and the reference-labelled
    Schnorr tuples (bad keys, off-curve x, R at infinity, odd y(R), mutated s / e)."""
    ts = bip340_vectors() + schnorr_tuples()
    bad = [(t["cls"], t["verdict"]) for t in ts
           if lane.lane_schnorr_verify_twist(t["sig"], t["msg"], t["pub"]) != t["verdict"]]
    assert not bad, bad[:10]


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_lane_schnorr_signer_vs_reference(lane):
    """The generator's BIP340 signer (synthetic C5 inputs) produces signatures the reference
    accepts, for the x-only key the reference derives."""
    R = Reference()
    rng = random.Random(5)
    for i in range(40):
        d = rng.randrange(1, N).to_bytes(32, "big")
        k = rng.randrange(1, N).to_bytes(32, "big")
        msg = rng.randbytes(32)
        sig, xo = ctypes.create_string_buffer(64), ctypes.create_string_buffer(32)
        assert lane.lane_schnorr_sign(d, msg, k, sig, xo) == 1
        assert R.schnorr_verify(sig.raw, msg, xo.raw) == 1
        assert R.schnorr_sign(d, msg, bytes(32))[1] == xo.raw


TWIST_FORMS = ["lane_verify_twist", "lane_verify_twist_host"]  # SIMT lane code / host engine's form


@pytest.mark.parametrize("fn", TWIST_FORMS)
def test_lane_twist_matches_reference_fixtures(lane, fn):
    """The square-root-free path (csrc/ecdsa_twist.h) on every fixture tuple: compressed keys
    never decompressed, the key's y recovered as -alpha / beta; exceptional classes (R at
    infinity, x(A) == x(B), u1 == 0) take the exact fallback.  Both forms: the kernels' fixed-window
    lane code and the host engine's (wNAF Q half, variable-time inverses)."""
    O = Oracle()
    bad = []
    classes = {}
    for t in ecdsa_tuples():
        tag, x, y = pub_to_tuple(t["pub"])
        ok, r, s = O.der_parse_lax(t["sig"])
        if not ok:
            r = s = bytes(32)
        got = getattr(lane, fn)(tag, x, y, r, s, t["hash"])
        classes[t["cls"]] = classes.get(t["cls"], 0) + 1
        if got != t["verdict"]:
            bad.append((t["cls"], got, t["verdict"]))
    assert not bad, bad[:10]
    assert len(classes) > 10


def _der(r, s):
    def enc(v):
        b = v.to_bytes(32, "big").lstrip(b"\0") or b"\0"
        if b[0] & 0x80:
            b = b"\0" + b
        return b"\x02" + bytes([len(b)]) + b
    body = enc(r) + enc(s)
    return b"\x30" + bytes([len(body)]) + body


@pytest.mark.parametrize("fn", TWIST_FORMS)
def test_lane_twist_random_vs_oracle(lane, fn):
    """Random signed tuples with mutations (flipped key parity, random x -- about half of them
    non-residues --, hybrid / uncompressed encodings, negated y, message and s flips) through
    the square-root-free lane code against the oracle's CPubKey::Verify."""
    O = Oracle()
    rng = random.Random(11)
    P = 2**256 - 2**32 - 977
    bad, seen = [], set()
    for i in range(240):
        d = rng.randrange(1, N)
        msg = rng.randbytes(32)
        qx, qy = (int.from_bytes(b, "big") for b in O.ecmult_gen(d.to_bytes(32, "big")))
        k = rng.randrange(1, N)
        rx = int.from_bytes(O.ecmult_gen(k.to_bytes(32, "big"))[0], "big")
        r = rx % N
        s = pow(k, N - 2, N) * (int.from_bytes(msg, "big") % N + r * d) % N
        mode = i % 8
        comp = mode in (0, 1, 2, 3)
        if mode == 1:
            qy = P - qy                      # flipped parity: the signature is for -Q
        elif mode == 2:
            qx = rng.randrange(P)            # random x: non-residue about half the time
        elif mode == 3 or mode == 6:
            msg = bytes([msg[0] ^ 1]) + msg[1:]
        elif mode == 4:
            s = N - s                        # high s: normalised, still valid
        elif mode == 5:
            qy = P - qy                      # uncompressed, wrong y sign
        if comp:
            pub = bytes([2 + (qy & 1)]) + qx.to_bytes(32, "big")
        else:
            tag = rng.choice([4, 6 + (qy & 1)])
            pub = bytes([tag]) + qx.to_bytes(32, "big") + qy.to_bytes(32, "big")
        exp = O.pubkey_verify(pub, msg, _der(r, s))
        tag, x, y = pub_to_tuple(pub)
        got = getattr(lane, fn)(tag, x, y, r.to_bytes(32, "big"), s.to_bytes(32, "big"), msg)
        seen.add((mode, exp))
        if got != exp:
            bad.append((i, mode, got, exp))
    assert not bad, bad[:10]
    assert {(0, 1), (1, 0), (2, 0), (4, 1), (5, 0), (7, 1)} <= seen


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_lane_schnorr_twist_random_vs_reference(lane):
    """Random BIP340 signatures (the generator's signer) with mutations -- s, e (message), r,
    the key's x (a non-residue about half the time) -- through the square-root-free lane code
    against the reference's secp256k1_schnorrsig_verify."""
    R = Reference()
    rng = random.Random(23)
    bad, seen = [], set()
    for i in range(160):
        d = rng.randrange(1, N).to_bytes(32, "big")
        k = rng.randrange(1, N).to_bytes(32, "big")
        msg = rng.randbytes(32)
        sig, xo = ctypes.create_string_buffer(64), ctypes.create_string_buffer(32)
        assert lane.lane_schnorr_sign(d, msg, k, sig, xo) == 1
        sig, xo = bytearray(sig.raw), bytearray(xo.raw)
        mode = i % 5
        if mode == 1:
            sig[40] ^= 4
        elif mode == 2:
            msg = bytes([msg[0] ^ 1]) + msg[1:]
        elif mode == 3:
            sig[5] ^= 1
        elif mode == 4:
            xo = bytearray(rng.randbytes(32))
        sig, xo = bytes(sig), bytes(xo)
        exp = R.schnorr_verify(sig, msg, xo)
        got = lane.lane_schnorr_verify_twist(sig, msg, xo)
        seen.add((mode, exp))
        if got != exp:
            bad.append((i, mode, got, exp))
    assert not bad, bad[:10]
    assert (0, 1) in seen and (1, 0) in seen


def test_lane_scalar_mul_inv_mod_n(lane):
    """sc_mul / sc_inv (the mod-n product-scanning reduction) against Python integers: random
    operands, the edge values 0, 1, n - 1, n - 2 and operands just below 2^256 (reduced inputs
    are < n, but the fold must hold for any 512-bit product)."""
    rnd = random.Random(0x5C)
    edge = [0, 1, 2, N - 1, N - 2, (1 << 255), N >> 1, (1 << 256) - 1]
    pairs = [(a, b) for a in edge for b in edge]
    pairs += [(rnd.getrandbits(256), rnd.getrandbits(256)) for _ in range(3000)]
    out = ctypes.create_string_buffer(32)
    for a, b in pairs:
        lane.lane_sc_mul(a.to_bytes(32, "big"), b.to_bytes(32, "big"), out)
        assert int.from_bytes(out.raw, "big") == (a * b) % N, (hex(a), hex(b))
    for _ in range(200):
        a = rnd.randrange(1, N)
        lane.lane_sc_inv(a.to_bytes(32, "big"), out)
        assert int.from_bytes(out.raw, "big") == pow(a, -1, N)


def test_mi30_safegcd_inverse_host(lane):
    """The GPU lanes' inverse (csrc/modinv_device.h, compiled here for the CPU) against
    pow(a, -1, m) for p and n: edge and random operands (the device run is in test_field_gpu)."""
    P = 2**256 - 2**32 - 977
    rng = random.Random(0x30)
    arr = ctypes.c_uint32 * 8
    for m in (P, N):
        minv = pow(m, -1, 2**30)
        vals = [0, 1, 2, 3, m - 1, m - 2, (m + 1) // 2, 2**255 % m, 2**128] + \
            [rng.randrange(m) for _ in range(3000)]
        for a in vals:
            out = arr()
            lane.lane_mi30_inverse(arr(*[(a >> (32 * i)) & 0xFFFFFFFF for i in range(8)]),
                                   arr(*[(m >> (32 * i)) & 0xFFFFFFFF for i in range(8)]),
                                   ctypes.c_uint32(minv), out)
            got = sum(out[i] << (32 * i) for i in range(8))
            assert got == (pow(a, -1, m) if a else 0), (hex(m), hex(a))
