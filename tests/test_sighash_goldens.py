"""The reference's signature-hash goldens through the engine's sighash job builder and the GPU
sighash kernels (reference interpreter.cpp:1273-1364, 1366-1397,
1576-1642).

Three golden sets, all with the REFERENCE's sighashes:
* sighash_legacy.json: the 500 rows of the reference's own src/test/data/sighash.json
  (sighash_tests.cpp:162-210): random 32-bit hash types, NONE / SINGLE / ANYONECANPAY, the SINGLE
  bug, OP_CODESEPARATORs in the scriptCode;
* sighash_random.json.gz (make_sighash_random.py): 1,200 random legacy and BIP143 checks, the
  expected sighash from the reference's CheckECDSASignature -> SignatureHash;
* sighash_rows.json.gz (make_sighash_rows.py): the sighashes the reference's interpreter computed
  for the script-level goldens (script_tests.json / tx_valid.json / tx_invalid.json), compared with
  the msg rows of the engine's staged first round (the path bench.py times).

Each check is built by bcc_debug_sighash exactly as the deferring checker builds a deferred tuple's
job (host/engine.cpp add_sighash_job): legacy SIGHASH_ALL -> template job (K3'), other legacy types
-> host preimage (K3), the SINGLE bug -> ONE, BIP143 -> raw-tx job (K_wtx + K_win), BIP143 SINGLE
-> host preimage + aux messages (K1 + K2 + K3).  The CPU tests run the same job builder with the
device stage replaced by the oracle (tests/native/engine_host_stub.cpp).
"""
import ctypes
import gzip
import json
import os
from collections import Counter

import pytest

from fixtures import load_json

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def legacy_checks():
    rows = load_json("sighash_legacy.json")
    assert len(rows) == 500
    return [(bytes.fromhex(r["tx"]), bytes.fromhex(r["script"]), r["nin"], r["hashtype"], 0, 0)
            for r in rows], [r["sighash_raw"] for r in rows]


def random_checks():
    d = json.load(gzip.open(os.path.join(GOLDEN, "sighash_random.json.gz")))
    txs = [bytes.fromhex(t) for t in d["txs"]]
    cs = d["checks"]
    return [(txs[c["tx"]], bytes.fromhex(c["code"]), c["nin"], c["hashtype"], c["amount"],
             c["sigversion"]) for c in cs], [c["sighash_raw"] for c in cs]


def kinds(checks):
    """Which device job kind each check becomes (engine.cpp add_sighash_job)."""
    out = Counter()
    for tx, code, nin, ht, amount, sv in checks:
        b = ht & 0x1f
        if sv == 0:
            out["legacy_template" if not (ht & 0x80) and b not in (2, 3) else "legacy_host"] += 1
        else:
            out["bip143_single" if b == 3 else "bip143_rawtx"] += 1
    return out


def stub_sighash(checks):
    import bitcoinconsensus_amd as B
    import engine_stub
    L = engine_stub.load()
    L.stub_debug_sighash.argtypes = [ctypes.POINTER(B.SighashCheck), ctypes.c_size_t,
                                     ctypes.c_char_p]
    n = len(checks)
    arr = (B.SighashCheck * n)()
    keep = []
    for i, (tx, code, nin, ht, amount, sv) in enumerate(checks):
        tb, cb = ctypes.create_string_buffer(tx, max(1, len(tx))), \
            ctypes.create_string_buffer(code, max(1, len(code)))
        keep += [tb, cb]
        ht &= 0xffffffff
        arr[i] = B.SighashCheck(ctypes.addressof(tb), len(tx), ctypes.addressof(cb), len(code), nin,
                                ht - (1 << 32) if ht >= 1 << 31 else ht, amount, sv)
    out = ctypes.create_string_buffer(32 * n)
    assert L.stub_debug_sighash(arr, n, out) == 0
    return [out.raw[32 * i:32 * i + 32] for i in range(n)]


def test_golden_sets_cover_every_job_kind():
    k = kinds(legacy_checks()[0] + random_checks()[0])
    assert min(k[x] for x in ("legacy_template", "legacy_host", "bip143_rawtx",
                              "bip143_single")) >= 100, k
    single_bug = sum(1 for tx, code, nin, ht, a, sv in legacy_checks()[0] if ht & 0x1f == 3)
    assert single_bug > 0


@pytest.mark.parametrize("which", ["legacy", "random"])
def test_job_builder_matches_reference_cpu(which):
    checks, exp = legacy_checks() if which == "legacy" else random_checks()
    got = stub_sighash(checks)
    bad = [i for i in range(len(checks)) if got[i].hex() != exp[i]]
    assert not bad, bad[:10]


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["legacy", "random"])
def test_gpu_sighash_kernels_match_reference(which):
    import bitcoinconsensus_amd as B
    checks, exp = legacy_checks() if which == "legacy" else random_checks()
    got = B.debug_sighash(checks)
    bad = [(i, kinds([checks[i]])) for i in range(len(checks)) if got[i].hex() != exp[i]]
    assert not bad, bad[:10]
    # one batch of everything together (job kinds interleaved in one device round)
    allc, alle = legacy_checks(), random_checks()
    got = B.debug_sighash(allc[0] + alle[0])
    assert [g.hex() for g in got] == allc[1] + alle[1]


@pytest.mark.gpu
def test_gpu_staged_sighash_rows_match_reference_interpreter():
    """The script-level goldens staged as the engine's first round (bcc_workload_from_items: the
    path bench.py times): for every case the sighashes the REFERENCE's interpreter computed (up to
    its first failing check) are among the msg rows the GPU wrote for that item."""
    import bitcoinconsensus_amd as B
    cases = json.load(gzip.open(os.path.join(GOLDEN, "script_cases.json.gz")))
    rows = json.load(gzip.open(os.path.join(GOLDEN, "sighash_rows.json.gz")))
    assert len(rows) >= 300 and sum(sum(r["sigversion"]) for r in rows) >= 100
    by_flags = {}
    for r in rows:
        by_flags.setdefault(cases[r["case"]]["flags"], []).append(r)
    checked = 0
    for flags, rs in by_flags.items():
        items = [(bytes.fromhex(cases[r["case"]]["spk"]), cases[r["case"]]["amount"],
                  bytes.fromhex(cases[r["case"]]["tx"]), cases[r["case"]]["nin"]) for r in rs]
        w = B.Workload(kind="items", items=items, flags=flags)
        try:
            w.run_sighash()
            msgs = w.msgs()
            owner = w.tuple_items()
        finally:
            w.free()
        per_item = [set() for _ in rs]
        for k, it in enumerate(owner):
            per_item[it].add(msgs[32 * k:32 * k + 32].hex())
        for j, r in enumerate(rs):
            # (a check repeated with the same key, signature and scriptCode is one row: the
            # engine asks the GPU once per distinct check)
            missing = set(r["sighash"]) - per_item[j]
            assert not missing, (cases[r["case"]]["src"], flags, missing)
            checked += len(r["sighash"])
    assert checked >= 400
