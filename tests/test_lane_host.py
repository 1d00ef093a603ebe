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
                    for f in ("ecdsa_lane.h", "secp256k1_device.h", "sha256_device.h")]
    if not os.path.exists(SO) or any(os.path.getmtime(d) > os.path.getmtime(SO) for d in deps):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO, src])
    return ctypes.CDLL(SO)


def test_lane_schnorr_matches_reference_fixtures(lane):
    ts = bip340_vectors() + schnorr_tuples()[::2]
    bad = [(t["cls"], lane.lane_schnorr_verify(t["sig"], t["msg"], t["pub"]), t["verdict"])
           for t in ts if lane.lane_schnorr_verify(t["sig"], t["msg"], t["pub"]) != t["verdict"]]
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


def test_lane_code_matches_reference_fixtures(lane):
    O = Oracle()
    ts = ecdsa_tuples()
    bad = []
    for i, t in enumerate(ts[::3]):  # every 3rd tuple keeps the CPU run short
        tag, x, y = pub_to_tuple(t["pub"])
        ok, r, s = O.der_parse_lax(t["sig"])
        if not ok:
            r = s = bytes(32)
        got = lane.lane_verify(tag, x, y, r, s, t["hash"])
        if got != t["verdict"]:
            bad.append((t["cls"], got, t["verdict"]))
    assert not bad, bad[:10]
