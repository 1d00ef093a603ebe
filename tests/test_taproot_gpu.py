"""GPU: BIP341/342 signature checks through the product C ABI (bcc_taproot_verify_batch:
csrc/host/taproot.cpp + sighash.hip tapsighash / aux kernels + the BIP340 kernels) against the
reference's CheckSchnorrSignature (interpreter.cpp:1678-1704): every committed case with its
sighash, and a fresh random batch (valid + mutated) checked item by item against oracle/_ref."""
import os
import random
import sys

import pytest

import bitcoinconsensus_amd as B
from fixtures import taproot_checks
from oracle_ctypes import Reference, reference_available
from test_taproot_host import check_against_golden

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_taproot_fixtures as G  # noqa: E402

pytestmark = pytest.mark.gpu


def test_taproot_golden_cases_on_gpu():
    cases = taproot_checks()
    out, hs = B.taproot_verify_batch(cases, sighashes=True)
    check_against_golden(out, hs, cases)


def test_taproot_golden_cases_sharded_on_gpu():
    """device = -1 over the configured devices (one here) gives the same results."""
    cases = taproot_checks()
    out, hs = B.taproot_verify_batch(cases, device=-1, sighashes=True)
    check_against_golden(out, hs, cases)


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_taproot_random_batch_vs_reference():
    R = Reference()
    rng = random.Random(0xB1B341)
    checks = []
    for k in range(3000):
        t = G.make_tx(rng, nout=rng.randrange(1, 4), long_ok=rng.random() < 0.2)
        nin = rng.randrange(len(t["vin"]))
        G.taproot_input(rng, t, nin)
        ht = rng.choice([0, 1, 2, 3, 0x81, 0x82, 0x83])
        if ht & 3 == 3 and nin >= len(t["vout"]):
            ht = 1
        sv = rng.randrange(2)
        annex = b"\x50" + rng.randbytes(rng.randrange(0, 120)) if rng.random() < 0.3 else None
        leaf, cpos = rng.randbytes(32), rng.choice([0xFFFFFFFF, rng.randrange(100)])
        tx, spent = G.tx_bytes(t), G.ser_outs(t["spent"])
        dummy = bytes(64) + (bytes([ht]) if ht else b"")
        _, _, h = R.taproot_check(tx, spent, nin, dummy, bytes(32), sv, annex, leaf, cpos)
        sig, pk = R.schnorr_sign(rng.randbytes(32), h, rng.randbytes(32))
        sig += bytes([ht]) if ht else b""
        c = dict(tx=tx, spent=spent, nin=nin, sig=sig, pk=pk, sigversion=sv, annex=annex,
                 tapleaf=leaf, codesep=cpos)
        r = rng.random()
        if r < 0.15:
            b = bytearray(sig)
            b[rng.randrange(64)] ^= 1 << rng.randrange(8)
            c["sig"] = bytes(b)
        elif r < 0.2:
            c["codesep"] ^= 1
        checks.append(c)
        # every input of a multi-input tx signed in turn shares the tx objects
        if rng.random() < 0.1:
            for j in range(len(t["vin"])):
                checks.append(dict(c, nin=j))
    out, hs = B.taproot_verify_batch(checks, sighashes=True)
    bad = []
    for i, c in enumerate(checks):
        ret, serr, h = R.taproot_check(c["tx"], c["spent"], c["nin"], c["sig"], c["pk"],
                                       c["sigversion"], c["annex"], c["tapleaf"], c["codesep"])
        if out[i][0] != ret or (ret == 0 and out[i][1] != serr) or (h is not None and hs[i] != h):
            bad.append((i, out[i], ret, serr))
    assert not bad, bad[:10]
    assert sum(o[0] == 1 for o in out) > 2000


def test_taproot_pipelined_rounds_equal_single_rounds():
    """A batch of at least two pipeline rounds (2 x 131,072 checks) runs as rounds alternating
    between two device contexts (one round's upload beside the previous round's kernels): every
    ret / serror / sighash equals the same checks run in single-round calls, the corrupted 5 % are
    exactly the invalid ones, and a sample matches the reference."""
    import ctypes
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n = 600_000
    job = bench.C5T(B, n, 0x5EED0106, 0)
    L = B.lib()
    ret = np.zeros(n, np.int32)
    err = np.zeros(n, np.int32)
    hs = np.zeros((n, 32), np.uint8)
    p32 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))  # noqa: E731
    assert L.bcc_taproot_verify_batch(job.arr, n, p32(ret), p32(err), hs.ctypes.data, 0) == 0
    ret1 = np.zeros(n, np.int32)
    err1 = np.zeros(n, np.int32)
    hs1 = np.zeros((n, 32), np.uint8)
    T = B.TaprootCheck
    step = 100_000  # each call below two pipeline rounds: a single round
    for lo in range(0, n, step):
        m = min(step, n - lo)
        arr = ctypes.cast(ctypes.addressof(job.arr) + lo * ctypes.sizeof(T), ctypes.POINTER(T))
        assert L.bcc_taproot_verify_batch(arr, m, p32(ret1[lo:]), p32(err1[lo:]),
                                          hs1[lo:].ctypes.data, 0) == 0
    assert np.array_equal(ret, ret1) and np.array_equal(err, err1) and np.array_equal(hs, hs1)
    assert int((ret == 1).sum()) == job.expect
    assert np.array_equal(hs, job.hs)  # the sighashes the signatures were made over
    if reference_available():
        R = Reference()
        for i in np.random.default_rng(5).choice(n, 300, replace=False):
            r, e, h = R.taproot_check(bytes(job.tx[i]), bytes(job.spent[i]), 0, bytes(job.sig[i]),
                                      bytes(job.xo[i]), 0)
            assert (r, e) == (int(ret[i]), int(err[i])) and h == bytes(hs[i]), i
