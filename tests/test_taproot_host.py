"""CPU: the product's BIP341/342 host front end (csrc/host/taproot.cpp: size / hash_type rules,
SigMsg serialization with digest slots, per-tx aux messages, parts + merge, device sharding) with
the device pipeline replaced by the oracle (tests/native/engine_host_stub.cpp), against the
reference's (ret, serror, sighash) on every committed case (tests/golden/taproot_checks.json.gz).
The -m gpu twin (test_taproot_gpu.py) runs the same cases through librbc_amd.so."""
import pytest

import bitcoinconsensus_amd as B
import engine_stub
from fixtures import taproot_checks


@pytest.fixture(scope="module")
def L():
    return engine_stub.load()


def check_against_golden(out, hs, cases):
    bad = []
    for i, ((ret, serr), h, c) in enumerate(zip(out, hs, cases)):
        if ret != c["ret"]:
            bad.append((i, c["cls"], "ret", ret, c["ret"]))
        elif ret == 0 and serr != c["serror"]:
            bad.append((i, c["cls"], "serror", serr, c["serror"]))
        elif ret == -1 and serr != 1:
            bad.append((i, c["cls"], "refused serror", serr))
        want = c["sighash"] if c["sighash"] is not None else bytes(32)
        if ret != -1 and h != want:
            bad.append((i, c["cls"], "sighash"))
    assert not bad, bad[:10]


def test_taproot_host_front_end_matches_reference(L):
    cases = taproot_checks()
    out, hs = B.taproot_verify_batch(cases, sighashes=True, library=L)
    check_against_golden(out, hs, cases)


def test_taproot_parts_merge_and_sharding(L):
    """> 2 x 2048 items: several host parts merged into one round; then the same batch spread
    over 3 'devices' (the stub ignores the id) must give identical results."""
    cases = taproot_checks() * 3
    out, hs = B.taproot_verify_batch(cases, sighashes=True, library=L)
    check_against_golden(out, hs, cases)
    try:
        engine_stub.set_devices(L, [0, 1, 2])
        out2, hs2 = B.taproot_verify_batch(cases, device=-1, sighashes=True, library=L)
    finally:
        engine_stub.set_devices(L, [])
    assert out2 == out and hs2 == hs


def test_taproot_null_and_empty(L):
    assert B.taproot_verify_batch([], library=L) == []
    c = dict(taproot_checks()[0])
    c["tx"] = b""
    assert B.taproot_verify_batch([c], library=L) == [(-1, 1)]
