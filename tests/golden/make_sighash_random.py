"""Random signature-hash checks with the REFERENCE's SignatureHash (run in the build container,
where oracle/_ref is built from /root/reference).

    python3 tests/golden/make_sighash_random.py

Each check is (tx, nIn, scriptCode, hash type byte, amount, sigversion) over random transactions:
1-8 inputs (a few with 253+ inputs / scripts, i.e. 3-byte compact sizes), 0-5 outputs, random
scriptSigs, sequences, versions and lock times, with and without BIP144 witnesses; scriptCodes of
0-300 bytes salted with OP_CODESEPARATOR (0xab); hash types ALL / NONE / SINGLE, each with and
without ANYONECANPAY, plus random bytes; SINGLE with nIn beyond the outputs (legacy: the ONE bug;
BIP143: hashOutputs = 0).  The expected sighash of every check is the reference's
(oracle/ref_shim.cpp ref_check_sighash: GenericTransactionSignatureChecker::CheckECDSASignature,
interpreter.cpp:1656-1676 -> SignatureHash, :1576-1642).
Output: sighash_random.json.gz = {"txs": [hex], "checks": [{"tx": index into txs, "nin", "code",
"hashtype", "amount", "sigversion", "sighash_raw"}]} (hex; sighash_raw = raw uint256 bytes, the
ECDSA message); PER_TX checks per transaction.
"""
import ctypes
import gzip
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_ctypes import Reference  # noqa: E402

N = 1200
PER_TX = 4
SEED = 0x5161A5


def compact(n):
    if n < 253:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + n.to_bytes(2, "little")
    return b"\xfe" + n.to_bytes(4, "little")


def rand_tx(rng):
    big = rng.random() < 0.012
    nin = rng.randint(253, 256) if big else rng.randint(1, 8)
    nout = rng.randint(0, 5)
    witness = rng.random() < 0.4
    out = bytearray(rng.getrandbits(32).to_bytes(4, "little"))
    if witness:
        out += b"\x00\x01"
    out += compact(nin)
    for _ in range(nin):
        out += rng.randbytes(36)
        ln = rng.choice([0, 0, 0, rng.randint(1, 110), rng.randint(200, 300)]) if not big else 0
        out += compact(ln) + rng.randbytes(ln)
        out += rng.choice([b"\xff\xff\xff\xff", rng.randbytes(4)])
    out += compact(nout)
    for _ in range(nout):
        out += rng.randbytes(8)
        ln = rng.choice([22, 25, 34, rng.randint(0, 80), rng.randint(0, 80), rng.randint(253, 260)])
        out += compact(ln) + rng.randbytes(ln)
    if witness:
        for _ in range(nin):
            k = rng.randint(1, 3)  # every stack non-empty: no superfluous-witness rejection
            out += compact(k)
            for _ in range(k):
                ln = rng.randint(0, 80)
                out += compact(ln) + rng.randbytes(ln)
    out += rng.getrandbits(32).to_bytes(4, "little")
    return bytes(out), nin, nout


def main():
    R = Reference()
    R.L.ref_check_sighash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint,
                                      ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint,
                                      ctypes.c_int64, ctypes.c_int, ctypes.c_char_p]
    rng = random.Random(SEED)
    rows, txs = [], []
    while len(rows) < N:
        if len(rows) % PER_TX == 0:
            tx, nin, nout = rand_tx(rng)
            txs.append(tx.hex())
        k = rng.randrange(nin)
        if rng.random() < 0.15 and nin > nout:
            k = rng.randrange(nout, nin)  # SINGLE beyond the outputs
        ln = rng.choice([0, 25, rng.randint(1, 80), rng.randint(240, 300)])
        code = bytearray(rng.randbytes(ln))
        for _ in range(rng.choice([0, 0, 1, 3])):
            if code:
                code[rng.randrange(len(code))] = 0xAB  # OP_CODESEPARATOR
        base = rng.choice([1, 2, 3])
        ht = rng.choice([base, base | 0x80, rng.randrange(256)])
        sv = rng.randrange(2)
        amount = rng.choice([0, rng.randrange(1 << 51), rng.getrandbits(64) - (1 << 63)])
        h = ctypes.create_string_buffer(32)
        r = R.L.ref_check_sighash(tx, len(tx), k, bytes(code), len(code), ht, amount, sv, h)
        assert r == 1, (tx.hex(), k)
        rows.append(dict(tx=len(txs) - 1, nin=k, code=bytes(code).hex(), hashtype=ht, amount=amount,
                         sigversion=sv, sighash_raw=h.raw.hex()))
    with gzip.open(os.path.join(HERE, "sighash_random.json.gz"), "wt") as fh:
        json.dump(dict(txs=txs, checks=rows), fh)
    print(f"sighash_random: {len(rows)} checks "
          f"({sum(r['sigversion'] for r in rows)} BIP143, "
          f"{sum(1 for r in rows if r['hashtype'] & 0x1f == 3)} SINGLE)")


if __name__ == "__main__":
    main()
