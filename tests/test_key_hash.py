"""The HASH160(pubkey) == program check of key-hash spends taken over by the device
(bcc_set_device_key_hash; csrc/host/engine.cpp DeferringChecker::defer_key_hash, sighash.hip
key_hash_kernel): spends whose signature is VALID for the key they carry but whose key hashes to
another program — only the key-hash check can reject them (the reference stops at OP_EQUALVERIFY,
interpreter.cpp:871-884 for P2PKH, :1936-1945 for P2WPKH) — beside the same spends with the right
program, for P2WPKH, P2SH-P2WPKH and P2PKH with compressed, uncompressed and hybrid keys.

Verdicts come from the reference library (oracle/_ref) on the same items.  CPU: the engine's host
logic with the stub device (tests/native/engine_host_stub.cpp applies the rows' key-hash
conditions the way the kernel does); GPU: librbc_amd.so."""
import ctypes
import hashlib
import struct

import pytest

import engine_stub
from oracle_ctypes import Oracle, Reference, reference_available
from script_asm import _ripemd160, hash160, push_data, ser_tx

VERIFY_ALL = 0xE15  # P2SH | DERSIG | NULLDUMMY | CHECKLOCKTIMEVERIFY | CHECKSEQUENCEVERIFY | WITNESS

needs_ref = pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")


def test_python_ripemd160_vectors():
    """The test's own RIPEMD-160 against the published vectors (Dobbertin-Bosselaers-Preneel)."""
    assert _ripemd160(b"").hex() == "9c1185a5c5e9fc54612808977ee8f548b2258d31"
    assert _ripemd160(b"abc").hex() == "8eb208f7e05d987a9b044a8e98c6b087f15a0bfc"
    assert _ripemd160(b"1234567890" * 8).hex() == "9b752e45573d4b39f4dbd3323cab82bf63326bfb"


def key_hash_items():
    """[(spk, amount, tx, nin, label)]: every (kind, key form, right / wrong program) once."""
    R, O = Reference(), Oracle()
    ska = hashlib.sha256(b"key-hash a").digest()
    skb = hashlib.sha256(b"key-hash b").digest()
    out = []
    n = 0
    for kind in ("p2wpkh", "p2sh_p2wpkh", "p2pkh"):
        for form in ("compressed", "uncompressed", "hybrid"):
            for wrong in (False, True):
                n += 1
                pa = R.pubkey_create(ska, form == "compressed")
                pb = R.pubkey_create(skb, form == "compressed")
                if form == "hybrid":  # 0x06 / 0x07 with y's parity (libsecp256k1 parses it)
                    pa = bytes([6 | (pa[64] & 1)]) + pa[1:]
                    pb = bytes([6 | (pb[64] & 1)]) + pb[1:]
                prog = hash160(pb if wrong else pa)
                amount = 100000 + n
                prevout = hashlib.sha256(b"prevout %d" % n).digest() + struct.pack("<I", n % 3)
                outs = [(amount - 1000, b"\x51")]
                p2pkh_code = b"\x76\xa9\x14" + prog + b"\x88\xac"
                if kind == "p2pkh":
                    spk = p2pkh_code
                    bare = ser_tx(1, [(prevout, b"", 0xFFFFFFFF)], outs, 0)
                    h = O.sighash(bare, 0, spk, 1, amount, 0)
                    sig = R.sign(ska, h) + b"\x01"
                    tx = ser_tx(1, [(prevout, push_data(sig) + push_data(pa), 0xFFFFFFFF)], outs, 0)
                else:
                    wprog = b"\x00\x14" + prog
                    if kind == "p2wpkh":
                        spk, ss = wprog, b""
                    else:
                        spk = b"\xa9\x14" + hash160(wprog) + b"\x87"
                        ss = push_data(wprog)
                    bare = ser_tx(1, [(prevout, ss, 0xFFFFFFFF)], outs, 0)
                    h = O.sighash(bare, 0, p2pkh_code, 1, amount, 1)
                    sig = R.sign(ska, h) + b"\x01"
                    tx = ser_tx(1, [(prevout, ss, 0xFFFFFFFF)], outs, 0, [[sig, pa]])
                out.append((spk, amount, tx, 0, (kind, form, wrong)))
    return out


def expected(items):
    R = Reference()
    exp = [R.verify_script_with_amount(s, a, t, i, VERIFY_ALL) for s, a, t, i, _ in items]
    for (_, _, _, _, lab), e in zip(items, exp):
        assert e[0] == (0 if lab[2] else 1), (lab, e)  # the construction does what it says
    return exp


class _Item(ctypes.Structure):
    _fields_ = [("script_pubkey", ctypes.c_void_p), ("script_pubkey_len", ctypes.c_uint),
                ("amount", ctypes.c_int64), ("tx_to", ctypes.c_void_p),
                ("tx_to_len", ctypes.c_uint), ("n_in", ctypes.c_uint)]


def _stub_batch(L, items):
    keep, arr = [], (_Item * len(items))()
    for k, (spk, amt, tx, nin) in enumerate(items):
        bs = ctypes.create_string_buffer(spk, len(spk))
        bt = ctypes.create_string_buffer(tx, len(tx))
        keep += [bs, bt]
        arr[k] = _Item(ctypes.addressof(bs), len(spk), amt, ctypes.addressof(bt), len(tx), nin)
    ret = (ctypes.c_int * len(items))()
    err = (ctypes.c_int * len(items))()
    L.bitcoinconsensus_verify_batch(arr, len(items), VERIFY_ALL, ret, err)
    return list(zip(ret, err))


@needs_ref
@pytest.mark.parametrize("on", [1, 0])
def test_key_hash_stub(on):
    L = engine_stub.load()
    L.bcc_set_device_key_hash.argtypes = [ctypes.c_int]
    items = key_hash_items()
    exp = expected(items)
    plain = [it[:4] for it in items]
    try:
        L.bcc_set_device_key_hash(on)
        # each item alone, and all of them (twice over) in one batch
        for it, e in zip(plain, exp):
            assert _stub_batch(L, [it]) == [e]
        assert _stub_batch(L, plain * 2) == exp * 2
    finally:
        L.bcc_set_device_key_hash(1)


@needs_ref
@pytest.mark.gpu
@pytest.mark.parametrize("on", [1, 0])
def test_key_hash_gpu(on):
    import bitcoinconsensus_amd as B
    items = key_hash_items()
    exp = expected(items)
    plain = [it[:4] for it in items]
    try:
        B.set_device_key_hash(on)
        for it, e in zip(plain, exp):
            got = B.verify_batch([it])
            assert [(r, int(x)) for r, x in got] == [e], it
        got = B.verify_batch(plain * 4)
        assert [(r, int(x)) for r, x in got] == exp * 4
        st = B.last_batch_stats()
        # on: every key-hash spend's first run carried its condition to the device (the hybrid
        # P2PKH / P2WPKH spends too); off: none did
        assert (st["device_key_hashes"] == 4 * len(items)) == bool(on), st["device_key_hashes"]
        assert (st["device_key_hashes"] == 0) == (not on)
    finally:
        B.set_device_key_hash(1)
