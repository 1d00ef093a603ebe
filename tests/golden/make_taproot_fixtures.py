"""Generate tests/golden/taproot_checks.json.gz (run in the build container, where the reference exists).

    python3 tests/golden/make_taproot_fixtures.py

BIP341 / BIP342 signature checks, GenericTransactionSignatureChecker::CheckSchnorrSignature
(depend/bitcoin/src/script/interpreter.cpp:1678-1704) over SignatureHashSchnorr (:1491-1574) with
the tx's PrecomputedTransactionData initialised from its spent outputs (:1422-1472).  The reference
ships no BIP341 vectors, so the cases are synthetic; every expected (ret, serror, sighash) comes
from the REFERENCE (oracle/_ref/libref_consensus.so via ref_shim.cpp's ref_taproot_check), never
from how the case was built.  Signatures are made with the reference's secp256k1_schnorrsig_sign
over the sighash the reference computed.

Case classes: every valid hash_type (0 with a 64-byte sig, 1-3, 0x81-0x83) x key path / tapscript
x annex absent / present (short and multi-block) x short / long spent scripts (multi-block
ANYONECANPAY messages), SIGHASH_SINGLE without a matching output, invalid hash_types, sig sizes
other than 64/65, 65-byte sigs with hash_type 0, flipped signature / key / tx-field bytes, keys that
do not parse, and inputs the checker refuses (spent-output count mismatch, index out of range).
"""
import gzip
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_ctypes import Reference  # noqa: E402

OUT = os.path.join(HERE, "taproot_checks.json.gz")


def cs(n):
    if n < 253:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + n.to_bytes(2, "little")
    return b"\xfe" + n.to_bytes(4, "little")


def ser_tx(version, vin, vout, locktime, witness=None):
    """vin: [(prevout36, scriptSig, seq)], vout: [(value, script)], witness: [[items]] or None."""
    out = version.to_bytes(4, "little", signed=True)
    if witness is not None:
        out += b"\x00\x01"
    out += cs(len(vin))
    for prev, ss, seq in vin:
        out += prev + cs(len(ss)) + ss + seq.to_bytes(4, "little")
    out += cs(len(vout))
    for v, spk in vout:
        out += v.to_bytes(8, "little", signed=True) + cs(len(spk)) + spk
    if witness is not None:
        for st in witness:
            out += cs(len(st)) + b"".join(cs(len(x)) + x for x in st)
    return out + locktime.to_bytes(4, "little")


def ser_outs(outs):
    return cs(len(outs)) + b"".join(v.to_bytes(8, "little", signed=True) + cs(len(s)) + s
                                    for v, s in outs)


def rand_script(rng, long_ok):
    k = rng.random()
    if k < 0.5:
        return b"\x51\x20" + rng.randbytes(32)           # P2TR
    if k < 0.7:
        return b"\x00\x14" + rng.randbytes(20)           # P2WPKH
    if k < 0.85 or not long_ok:
        return rng.randbytes(rng.randrange(0, 80))
    return rng.randbytes(rng.randrange(200, 700))        # multi-block ACP messages


def make_tx(rng, nin=None, nout=None, long_ok=True):
    nin = nin if nin is not None else rng.randrange(1, 6)
    nout = nout if nout is not None else rng.randrange(0, 5)
    vin = [(rng.randbytes(32) + rng.randrange(0, 5).to_bytes(4, "little"),
            rng.randbytes(rng.randrange(0, 3)) if rng.random() < 0.2 else b"",
            rng.choice([0xFFFFFFFF, 0xFFFFFFFE, rng.getrandbits(32)])) for _ in range(nin)]
    vout = [(rng.randrange(0, 21_000_000 * 10**8), rand_script(rng, long_ok)) for _ in range(nout)]
    wit = [[rng.randbytes(64)] for _ in range(nin)] if rng.random() < 0.7 and nin else None
    version = rng.choice([1, 2, -1, rng.getrandbits(31)])
    locktime = rng.choice([0, rng.getrandbits(32)])
    spent = [(rng.randrange(0, 21_000_000 * 10**8), rand_script(rng, long_ok)) for _ in range(nin)]
    return dict(version=version, vin=vin, vout=vout, locktime=locktime, wit=wit, spent=spent)


def taproot_input(rng, t, nin):
    """Make input nin a key/script-path Taproot spend: a witness and a P2TR spent output (what
    PrecomputedTransactionData::Init needs to be BIP341-ready, interpreter.cpp:1436-1452)."""
    if t["wit"] is None:
        t["wit"] = [[] for _ in t["vin"]]
    t["wit"] = list(t["wit"])
    t["wit"][nin] = [rng.randbytes(64)]
    t["spent"] = list(t["spent"])
    t["spent"][nin] = (t["spent"][nin][0], b"\x51\x20" + rng.randbytes(32))
    return t


def tx_bytes(t):
    return ser_tx(t["version"], t["vin"], t["vout"], t["locktime"], t["wit"])


def main():
    R = Reference()
    rng = random.Random(0x7A9_5EED)
    cases = []

    def emit(tx, spent, nin, sig, pk, sv, annex, leaf, cpos, cls):
        ret, serr, h = R.taproot_check(tx, spent, nin, sig, pk, sv, annex, leaf, cpos)
        cases.append(dict(cls=cls, tx=tx.hex(), spent=spent.hex(), nin=nin, sig=sig.hex(),
                          pk=pk.hex(), sigversion=sv, annex=None if annex is None else annex.hex(),
                          tapleaf=leaf.hex(), codesep=cpos, ret=ret, serror=serr,
                          sighash=None if h is None else h.hex()))
        return ret, h

    def signed(t, nin, ht, sv, annex, leaf, cpos, sk):
        tx, spent = tx_bytes(t), ser_outs(t["spent"])
        dummy = bytes(64) + (bytes([ht]) if ht else b"")
        _, _, h = R.taproot_check(tx, spent, nin, dummy, bytes(32), sv, annex, leaf, cpos)
        if h is None:
            return None
        sig, pk = R.schnorr_sign(sk, h, rng.randbytes(32))
        return tx, spent, sig + (bytes([ht]) if ht else b""), pk

    hts = [0, 1, 2, 3, 0x81, 0x82, 0x83]
    # valid signatures over the full grid (plus random txs)
    for ht in hts:
        for sv in (0, 1):
            for ak in ("none", "short", "long"):
                for rep in range(3):
                    t = make_tx(rng, nout=rng.randrange(1, 5))
                    nin = rng.randrange(len(t["vin"]))
                    taproot_input(rng, t, nin)
                    if ht & 3 == 3 and nin >= len(t["vout"]):
                        t["vout"] += [(1000, b"\x51")] * (nin + 1 - len(t["vout"]))
                    annex = None if ak == "none" else b"\x50" + rng.randbytes(
                        rng.randrange(0, 40) if ak == "short" else rng.randrange(100, 400))
                    leaf = rng.randbytes(32)
                    cpos = rng.choice([0xFFFFFFFF, rng.randrange(0, 200)])
                    sk = rng.randbytes(32)
                    r = signed(t, nin, ht, sv, annex, leaf, cpos, sk)
                    assert r is not None
                    tx, spent, sig, pk = r
                    ret, _ = emit(tx, spent, nin, sig, pk, sv, annex, leaf, cpos, "valid")
                    assert ret == 1
                    # mutations of the same check
                    k = rng.randrange(len(sig) if len(sig) == 64 else 64)
                    bad = bytearray(sig)
                    bad[k] ^= 1 << rng.randrange(8)
                    emit(tx, spent, nin, bytes(bad), pk, sv, annex, leaf, cpos, "sig_flip")
                    bpk = bytearray(pk)
                    bpk[rng.randrange(32)] ^= 1
                    emit(tx, spent, nin, sig, bytes(bpk), sv, annex, leaf, cpos, "pk_flip")
                    # a signed field changes: locktime (always hashed), the leaf / annex / an
                    # output amount (hashed or not depending on hash_type / sigversion)
                    t2 = dict(t)
                    t2["locktime"] = t["locktime"] ^ 1
                    emit(tx_bytes(t2), spent, nin, sig, pk, sv, annex, leaf, cpos, "locktime")
                    emit(tx, spent, nin, sig, pk, sv, annex, bytes(32), cpos ^ 1, "leaf_cpos")
                    emit(tx, spent, nin, sig, pk, 1 - sv, annex, leaf, cpos, "sigversion")
                    emit(tx, spent, nin, sig, pk, sv, None if annex else b"\x50", leaf, cpos,
                         "annex_toggle")
                    sp2 = list(t["spent"])
                    j = rng.randrange(len(sp2))
                    sp2[j] = (sp2[j][0] + 1, sp2[j][1])
                    emit(tx, ser_outs(sp2), nin, sig, pk, sv, annex, leaf, cpos, "spent_amount")
                    if t["vout"]:
                        t3 = dict(t)
                        t3["vout"] = list(t["vout"])
                        o = rng.randrange(len(t3["vout"]))
                        t3["vout"][o] = (t3["vout"][o][0] ^ 1, t3["vout"][o][1])
                        emit(tx_bytes(t3), spent, nin, sig, pk, sv, annex, leaf, cpos, "output")
                    # the hash_type byte rewritten after signing
                    if len(sig) == 65:
                        for nh in (0, 4, 0x80, 0x84, 0xFF, (ht ^ 0x80) if ht != 0x80 else 1):
                            emit(tx, spent, nin, sig[:64] + bytes([nh]), pk, sv, annex, leaf, cpos,
                                 "hashtype_byte")
                    else:
                        emit(tx, spent, nin, sig + b"\x01", pk, sv, annex, leaf, cpos,
                             "hashtype_added")
    # SIGHASH_SINGLE with nIn >= vout.size(); sig sizes; unparsable keys; refused inputs
    for _ in range(24):
        t = make_tx(rng, nin=rng.randrange(2, 5), nout=rng.randrange(0, 2))
        taproot_input(rng, t, 0)
        tx, spent = tx_bytes(t), ser_outs(t["spent"])
        nin = len(t["vin"]) - 1
        pk = R.schnorr_sign(rng.randbytes(32), bytes(32), bytes(32))[1]
        for ht in (3, 0x83):
            emit(tx, spent, nin, rng.randbytes(64) + bytes([ht]), pk, rng.randrange(2), None,
                 rng.randbytes(32), 0xFFFFFFFF, "single_no_output")
        for L in (0, 1, 32, 63, 66, 72):
            emit(tx, spent, 0, rng.randbytes(L), pk, 0, None, bytes(32), 0xFFFFFFFF, "sig_size")
        emit(tx, spent, 0, rng.randbytes(64), b"\xff" * 32, 0, None, bytes(32), 0xFFFFFFFF,
             "pk_not_on_curve_or_ge_p")
        emit(tx, ser_outs(t["spent"][:-1]), 0, rng.randbytes(64), pk, 0, None, bytes(32),
             0xFFFFFFFF, "refused_spent_count")
        emit(tx, spent, len(t["vin"]), rng.randbytes(64), pk, 0, None, bytes(32), 0xFFFFFFFF,
             "refused_index")
        t4 = make_tx(rng, nin=2, nout=1)
        t4["wit"] = None
        emit(tx_bytes(t4), ser_outs(t4["spent"]), 0, rng.randbytes(64), pk, 0, None, bytes(32),
             0xFFFFFFFF, "refused_not_bip341_ready")
        emit(tx + b"\x00", spent, 0, rng.randbytes(64), pk, 0, None, bytes(32), 0xFFFFFFFF,
             "refused_tx_trailing")
    # a many-input tx (long sha_prevouts / sha_scriptpubkeys messages), all inputs checked
    t = make_tx(rng, nin=300, nout=3, long_ok=False)
    taproot_input(rng, t, 5)
    for nin in range(0, 300, 7):
        ht = rng.choice(hts if nin < 3 else [0, 1, 2, 0x81, 0x82])
        r = signed(t, nin, ht, 0, None, bytes(32), 0xFFFFFFFF, rng.randbytes(32))
        tx, spent, sig, pk = r
        emit(tx, spent, nin, sig, pk, 0, None, bytes(32), 0xFFFFFFFF, "many_inputs")

    # blobs (txs / spent-output vectors) stored once, cases refer to them by index
    blobs, index = [], {}
    for c in cases:
        for k in ("tx", "spent"):
            if c[k] not in index:
                index[c[k]] = len(blobs)
                blobs.append(c[k])
            c[k] = index[c[k]]
    with gzip.open(OUT, "wt") as f:
        json.dump(dict(source="oracle/_ref ref_taproot_check (reference CheckSchnorrSignature)",
                       serror_names={"44": "SCHNORR_SIG_SIZE", "45": "SCHNORR_SIG_HASHTYPE",
                                     "46": "SCHNORR_SIG"},
                       blobs=blobs, cases=cases), f, separators=(",", ":"))
    by = {}
    for c in cases:
        by.setdefault(c["cls"], [0, 0])
        by[c["cls"]][0 if c["ret"] == 1 else 1] += 1
    print(len(cases), "cases", by,
          os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
