"""Reference-captured signature hashes of the script-level golden cases (run in the build
container, where oracle/_ref is built from /root/reference).

    python3 tests/golden/make_sighash_rows.py

For every case of script_cases.json.gz (the reference's script_tests.json / tx_valid.json /
tx_invalid.json re-expressed as C-ABI inputs, see make_script_cases.py) the REFERENCE interpreter
runs once with a capturing checker (oracle/ref_shim.cpp ref_capture_script: every call of
GenericTransactionSignatureChecker::VerifyECDSASignature, interpreter.cpp:1644-1676, with the
sighash SignatureHash produced for it, interpreter.cpp:1576-1642).  Recorded per case: the
sighashes (raw uint256 bytes, the ECDSA message) of the checks the reference made, in order, up to
the first check whose verdict was false — exactly the checks the engine's first speculative
interpreter run defers as GPU tuples (every consulted check before it answered true, so both runs
took the same path).  Legacy (SIGHASH_ALL templates, NONE / SINGLE / ANYONECANPAY, the SINGLE bug,
OP_CODESEPARATOR, FindAndDelete) and BIP143 (P2WPKH, P2WSH, every hash type) rows are all in.
Output: sighash_rows.json.gz = [{"case": index into script_cases, "sighash": [hex, ...],
"sigversion": [0 legacy | 1 witness, ...]}]
"""
import gzip
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_ctypes import Reference  # noqa: E402


def main():
    R = Reference()
    cases = json.load(gzip.open(os.path.join(HERE, "script_cases.json.gz")))
    out = []
    nrec = {0: 0, 1: 0}
    for i, c in enumerate(cases):
        spk, tx = bytes.fromhex(c["spk"]), bytes.fromhex(c["tx"])
        if c["err"] != 0:
            continue
        r, serr, recs = R.capture_script(spk, c["amount"], tx, c["nin"], c["flags"])
        hs, svs = [], []
        for rec in recs:
            if not rec["verdict"]:
                break
            hs.append(rec["sighash"].hex())
            # witness v0 iff the spent script or its P2SH redeem script is a witness program
            svs.append(1 if has_witness(tx, c["nin"]) else 0)
        if hs:
            out.append(dict(case=i, sighash=hs, sigversion=svs))
            for s in svs:
                nrec[s] += 1
    with gzip.open(os.path.join(HERE, "sighash_rows.json.gz"), "wt") as fh:
        json.dump(out, fh)
    print(f"sighash_rows: {len(out)} cases, {nrec[0]} legacy + {nrec[1]} witness-input sighashes")


def has_witness(tx, nin):
    """Whether input nin carries a witness (BIP144 serialization; a rough sigversion label for
    the summary only, the test does not depend on it)."""
    if len(tx) < 6 or tx[4] != 0 or tx[5] != 1:
        return False
    o = 6

    def cs(o):
        b = tx[o]
        if b < 253:
            return b, o + 1
        k = {253: 2, 254: 4, 255: 8}[b]
        return int.from_bytes(tx[o + 1:o + 1 + k], "little"), o + 1 + k
    nvin, o = cs(o)
    for _ in range(nvin):
        o += 36
        ln, o = cs(o)
        o += ln + 4
    nvout, o = cs(o)
    for _ in range(nvout):
        o += 8
        ln, o = cs(o)
        o += ln
    for k in range(nvin):
        nw, o = cs(o)
        if k == nin:
            return nw > 0
        for _ in range(nw):
            ln, o = cs(o)
            o += ln
    return False


if __name__ == "__main__":
    main()
