"""CPU: the engine's HOST logic (tx parser, interpreter, deferring checker, sighash job builder,
re-run stitching; csrc/host/*.cpp) against the reference on the reference's own script / tx test
data (tests/golden/script_cases.json.gz) and the crate vectors.

The device pipeline is replaced by tests/native/engine_host_stub.cpp, which evaluates the host-built
jobs with the oracle -- test-only; the product library is exercised by the -m gpu twins of these
tests (test_consensus_gpu.py)."""
import ctypes
import gzip
import json
import os
import subprocess

import pytest

import engine_stub

from fixtures import load_json

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(HERE, "native", "_build", "engine_host.so")
HOST_CHAIN_BLOCKS_DEFAULT = 160  # engine.cpp g_host_chain_blocks


class Item(ctypes.Structure):
    _fields_ = [("script_pubkey", ctypes.c_void_p), ("script_pubkey_len", ctypes.c_uint),
                ("amount", ctypes.c_int64), ("tx_to", ctypes.c_void_p),
                ("tx_to_len", ctypes.c_uint), ("n_in", ctypes.c_uint)]


@pytest.fixture(scope="module")
def eng():
    import engine_stub
    return engine_stub.load()


def call(L, spk, amount, tx, nin, flags):
    e = ctypes.c_int(-1)
    r = L.bitcoinconsensus_verify_script_with_amount(spk, len(spk), ctypes.c_int64(amount), tx,
                                                     len(tx), nin, flags, ctypes.byref(e))
    return r, e.value


def test_crate_vectors(eng):
    for v in load_json("crate_vectors.json"):
        got = call(eng, bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"], v["flags"])
        assert got == (v["ret"], v["err"]), v["name"]


def test_verify_script_no_amount(eng):
    v = load_json("crate_vectors.json")[0]
    spk, tx = bytes.fromhex(v["spk"]), bytes.fromhex(v["tx"])
    e = ctypes.c_int(-1)
    assert eng.bitcoinconsensus_verify_script(spk, len(spk), tx, len(tx), 0, 0xE15, ctypes.byref(e)) == 0
    assert e.value == 4  # ERR_AMOUNT_REQUIRED
    assert eng.bitcoinconsensus_verify_script(spk, len(spk), tx, len(tx), 0, 0x205, ctypes.byref(e)) == 1
    assert e.value == 0
    assert eng.bitcoinconsensus_version() == 1


def cases():
    return json.load(gzip.open(os.path.join(HERE, "golden", "script_cases.json.gz"), "rt"))


def test_script_cases_single_calls(eng):
    bad = []
    for c in cases():
        got = call(eng, bytes.fromhex(c["spk"]), c["amount"], bytes.fromhex(c["tx"]), c["nin"], c["flags"])
        if got != (c["ret"], c["err"]):
            bad.append((c["src"], c["flags"], got, (c["ret"], c["err"])))
    assert not bad, bad[:10]


def test_script_cases_as_batches(eng, stats=None):
    """verify_batch per flag set == single calls (shared tx buffers parsed once)."""
    allc = cases()
    by_flags = {}
    for c in allc:
        by_flags.setdefault(c["flags"], []).append(c)
    for flags, cs in by_flags.items():
        keep, txbufs = [], {}
        arr = (Item * len(cs))()
        for i, c in enumerate(cs):
            spk, tx = bytes.fromhex(c["spk"]), bytes.fromhex(c["tx"])
            bs = ctypes.create_string_buffer(spk, max(1, len(spk)))
            bt = txbufs.setdefault(tx, ctypes.create_string_buffer(tx, max(1, len(tx))))
            keep.append(bs)
            arr[i] = Item(ctypes.addressof(bs), len(spk), c["amount"], ctypes.addressof(bt), len(tx), c["nin"])
        ret = (ctypes.c_int * len(cs))()
        err = (ctypes.c_int * len(cs))()
        nvalid = eng.bitcoinconsensus_verify_batch(arr, len(cs), flags, ret, err)
        exp = [(c["ret"], c["err"]) for c in cs]
        got = list(zip(ret, err))
        assert got == exp
        assert nvalid == sum(r for r, _ in exp)
        if stats is not None:
            st = Stats()
            eng.bcc_last_batch_stats(ctypes.byref(st))
            stats.append(st.host_hashed)


def test_script_cases_pipelined(eng):
    """The same batches cut into pipeline chunks of 97 items (chunk device rounds on the worker
    thread overlapping the next chunk's host pass), alone and over three devices: identical to the
    single calls; an injected device failure in a pipelined chunk is retried."""
    eng.bcc_set_pipeline_chunk.argtypes = [ctypes.c_size_t]
    try:
        eng.bcc_set_pipeline_chunk(97)
        test_script_cases_as_batches(eng)
        engine_stub.set_devices(eng, [0, 1, 2])
        test_script_cases_as_batches(eng)
        engine_stub.set_devices(eng, [])
        eng.bcc_debug_fail_device_rounds(1)
        test_script_cases_as_batches(eng)
    finally:
        engine_stub.set_devices(eng, [])
        eng.bcc_set_pipeline_chunk(0)


def test_long_tx_runs_cut_into_entries(eng):
    """Items arriving as long runs on one tx buffer (the inputs of a many-input tx): prepare cuts
    a run longer than a quarter of a shard into several TxEntry pieces (each parsed on its own,
    with its own template / aux slots) so the interpreter shards balance.  Every item's result
    equals the reference label, with the pieces in different shards."""
    allc = cases()
    flags = max({c["flags"] for c in allc}, key=lambda f: sum(c["flags"] == f for c in allc))
    cs = [c for c in allc if c["flags"] == flags][:20]
    R = 300
    arr = (Item * (len(cs) * R))()
    keep = []
    for k, c in enumerate(cs):
        spk, tx = bytes.fromhex(c["spk"]), bytes.fromhex(c["tx"])
        bs = ctypes.create_string_buffer(spk, max(1, len(spk)))
        bt = ctypes.create_string_buffer(tx, max(1, len(tx)))
        keep += [bs, bt]
        for r in range(R):
            arr[k * R + r] = Item(ctypes.addressof(bs), len(spk), c["amount"], ctypes.addressof(bt),
                                  len(tx), c["nin"])
    ret = (ctypes.c_int * len(arr))()
    err = (ctypes.c_int * len(arr))()
    eng.bitcoinconsensus_verify_batch(arr, len(arr), flags, ret, err)
    got = list(zip(ret, err))
    exp = [(c["ret"], c["err"]) for c in cs for _ in range(R)]
    assert got == exp


@pytest.mark.parametrize("blocks", [1, 2, 5])
def test_script_cases_host_hashed_chains(eng, blocks):
    """Checks whose SHA chain exceeds `blocks` blocks hashed on the host (legacy template and
    preimage jobs in the parallel pass, long-tx BIP143 checks inline): identical results, as
    batches and as single calls."""
    eng.bcc_set_host_chain_blocks.argtypes = [ctypes.c_uint]
    eng.bcc_set_host_bip143_blocks.argtypes = [ctypes.c_uint]
    try:
        eng.bcc_set_host_chain_blocks(blocks)
        eng.bcc_set_host_bip143_blocks(blocks)
        hashed = []
        test_script_cases_as_batches(eng, hashed)
        assert sum(hashed) > 0  # the offload ran
        if blocks == 1:
            test_script_cases_single_calls(eng)
            test_crate_vectors(eng)
    finally:
        eng.bcc_set_host_chain_blocks(HOST_CHAIN_BLOCKS_DEFAULT)
        eng.bcc_set_host_bip143_blocks(32)


@pytest.mark.parametrize("on", [0, 1])
def test_script_cases_key_hash_where(eng, on):
    """The HASH160(pubkey) == program check of P2WPKH / P2PKH spends on the device beside the
    signature (on: the stub applies the rows' key-hash conditions like key_hash_kernel; a false
    verdict re-runs the input with the host comparison) or on the host before the run (off):
    identical results, batched and single; the deferred path carried conditions."""
    eng.bcc_set_device_key_hash.argtypes = [ctypes.c_int]
    try:
        eng.bcc_set_device_key_hash(on)
        allc = cases()
        n = [0]

        def count():
            st = Stats()
            eng.bcc_last_batch_stats(ctypes.byref(st))
            n[0] += st.device_key_hashes

        by_flags = {}
        for c in allc:
            by_flags.setdefault(c["flags"], []).append(c)
        for flags, cs in by_flags.items():
            keep, arr = [], (Item * len(cs))()
            for i, c in enumerate(cs):
                spk, tx = bytes.fromhex(c["spk"]), bytes.fromhex(c["tx"])
                bs = ctypes.create_string_buffer(spk, max(1, len(spk)))
                bt = ctypes.create_string_buffer(tx, max(1, len(tx)))
                keep += [bs, bt]
                arr[i] = Item(ctypes.addressof(bs), len(spk), c["amount"], ctypes.addressof(bt), len(tx), c["nin"])
            ret = (ctypes.c_int * len(cs))()
            err = (ctypes.c_int * len(cs))()
            eng.bitcoinconsensus_verify_batch(arr, len(cs), flags, ret, err)
            assert list(zip(ret, err)) == [(c["ret"], c["err"]) for c in cs]
            count()
        assert (n[0] > 0) == bool(on)
        test_script_cases_single_calls(eng)
        test_crate_vectors(eng)
    finally:
        eng.bcc_set_device_key_hash(1)


@pytest.mark.parametrize("host_lane", [False, True])
def test_pubkey_verify_batch_front_end(eng, host_lane):
    """bcc_pubkey_verify_batch on the reference-labelled adversarial tuple fixtures.  host_lane:
    every round on the host lane code, i.e. the product's host front end (parse_rows: CPubKey
    length filter, lax DER, r/s == 0; the host_verify_rows curve code); else the device round
    (stubbed by the oracle's CPubKey::Verify over the same blob slices).  Offsets that are not
    non-decreasing anywhere (one tuple past the blob, one running backwards, or the whole call
    backwards) are an argument error: -1, so that no verdict depends on the round split."""
    from fixtures import ecdsa_tuples
    ts = ecdsa_tuples()

    def blob(parts):
        off = [0]
        for p in parts:
            off.append(off[-1] + len(p))
        return b"".join(parts), (ctypes.c_uint64 * len(off))(*off)

    pb, po = blob([t["pub"] for t in ts])
    sb, so = blob([t["sig"] for t in ts])
    msg = b"".join(t["hash"] for t in ts)
    out = ctypes.create_string_buffer(len(ts))
    eng.bcc_set_host_small_round.argtypes = [ctypes.c_size_t]
    eng.bcc_set_host_small_round(1 << 30 if host_lane else 0)
    try:
        assert eng.bcc_pubkey_verify_batch(pb, po, msg, sb, so, out, len(ts), 0) == 0
        bad = [(t["cls"], i) for i, t in enumerate(ts) if out.raw[i] != t["verdict"]]
        assert not bad, bad[:20]
        keep = po[10]
        po[10] = 1 << 40  # tuple 9 past the blob, tuple 10 backwards
        assert eng.bcc_pubkey_verify_batch(pb, po, msg, sb, so, out, len(ts), 0) == -1
        po[10] = keep
        keep = so[20]
        so[20] = so[19] - 1  # tuple 19 backwards
        assert eng.bcc_pubkey_verify_batch(pb, po, msg, sb, so, out, len(ts), 0) == -1
        so[20] = keep
        assert eng.bcc_pubkey_verify_batch(pb, po, msg, sb, so, out, len(ts), 0) == 0
        assert list(out.raw) == [t["verdict"] for t in ts]
        po[0], po[len(ts)] = 1, 0
        assert eng.bcc_pubkey_verify_batch(pb, po, msg, sb, so, out, len(ts), 0) == -1
    finally:
        eng.bcc_set_host_small_round(int(os.environ.get("BCC_HOST_SMALL_ROUND", "16")))


def _batch(eng, vs, flags=None):
    keep = []
    arr = (Item * len(vs))()
    for i, v in enumerate(vs):
        spk, tx = bytes.fromhex(v["spk"]), bytes.fromhex(v["tx"])
        bs = ctypes.create_string_buffer(spk, max(1, len(spk)))
        bt = ctypes.create_string_buffer(tx, max(1, len(tx)))
        keep += [bs, bt]
        arr[i] = Item(ctypes.addressof(bs), len(spk), v["amount"], ctypes.addressof(bt), len(tx), v["nin"])
    ret = (ctypes.c_int * len(vs))()
    err = (ctypes.c_int * len(vs))()
    f = vs[0]["flags"] if flags is None else flags
    rc = eng.bitcoinconsensus_verify_batch(arr, len(vs), f, ret, err)
    return rc, list(zip(ret, err))


def Stats():
    """The package's mirror of bcc_batch_stats (checked against the C layout by
    tests/test_abi_symbols.py), so the engine never writes past a stale copy."""
    import bitcoinconsensus_amd as B
    return B.BatchStats()


def test_device_failure_retried_once(eng):
    """One injected device failure: the round is re-run on a fresh batch, results unchanged."""
    vs = [v for v in load_json("crate_vectors.json") if v["flags"] == 0xE15]
    eng.bcc_debug_fail_device_rounds(1)
    rc, got = _batch(eng, vs)
    st = Stats()
    eng.bcc_last_batch_stats(ctypes.byref(st))
    assert got == [(v["ret"], v["err"]) for v in vs]
    assert rc == sum(v["ret"] for v in vs)
    assert st.device_retries == 1


def test_device_failure_never_reported_as_invalid(eng):
    """BCC_DEVICE_FAILURE_ERROR, two failures in a row: verify_batch returns -1; items whose
    verdict needed the device get ret 0 / BCC_ERR_DEVICE_FAILURE (6), never a consensus error;
    items decided on the host before the device (here: bad flags) keep their reference result."""
    vs = [v for v in load_json("crate_vectors.json") if v["flags"] == 0xE15]
    assert eng.bcc_set_device_failure_policy(1) == 0
    try:
        eng.bcc_debug_fail_device_rounds(2)
        rc, got = _batch(eng, vs)
        eng.bcc_debug_fail_device_rounds(0)
    finally:
        eng.bcc_set_device_failure_policy(0)
    assert rc == -1
    for v, (r, e) in zip(vs, got):
        assert r == 0
        if v["ret"] == 1:  # needed a signature verdict: no verdict, flagged
            assert e == 6, (v["name"], e)
        else:              # e.g. EQUALVERIFY fails before any CHECKSIG: decided on the host
            assert e in (6, v["err"]), (v["name"], e)
    rc, got = _batch(eng, vs, flags=0xE15 + 1)  # host-decided: INVALID_FLAGS, no device round
    assert rc == 0 and all(g == (0, 5) for g in got)


def test_device_failure_verified_on_host(eng):
    """The default policy (BCC_DEVICE_FAILURE_HOST): a round the device cannot deliver (a transient
    error twice, or one sticky error, which is not retried) is verified on the host with the
    engine's own code, and every item gets exactly the reference's result."""
    vs = [v for v in load_json("crate_vectors.json") if v["flags"] == 0xE15]
    exp = [(v["ret"], v["err"]) for v in vs]
    eng.bcc_debug_fail_device_rounds_code.argtypes = [ctypes.c_int, ctypes.c_int]
    eng.bcc_host_fallback_rounds.restype = ctypes.c_size_t
    before = eng.bcc_host_fallback_rounds()
    for inject, retries in ((lambda: eng.bcc_debug_fail_device_rounds(2), 1),
                            (lambda: eng.bcc_debug_fail_device_rounds_code(1, 719), 0)):
        inject()
        rc, got = _batch(eng, vs)
        eng.bcc_debug_fail_device_rounds(0)
        st = Stats()
        eng.bcc_last_batch_stats(ctypes.byref(st))
        assert got == exp
        assert rc == sum(v["ret"] for v in vs)
        assert st.device_retries == retries and st.host_rounds == 1
    assert eng.bcc_host_fallback_rounds() == before + 2
    # the script-level goldens with every device round failing (one batch per flag set)
    eng.bcc_debug_fail_device_rounds_code(1 << 20, 719)
    try:
        test_script_cases_as_batches(eng)
    finally:
        eng.bcc_debug_fail_device_rounds(0)


def test_small_rounds_on_host(eng):
    """bcc_set_host_small_round: rounds of at most that many checks run on the host CPU with the
    same results (every script-level golden, single calls and batches)."""
    eng.bcc_set_host_small_round.argtypes = [ctypes.c_size_t]
    try:
        eng.bcc_set_host_small_round(1 << 30)
        test_script_cases_as_batches(eng)
        vs = load_json("crate_vectors.json")
        for v in vs:
            got = call(eng, bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"],
                       v["flags"])
            assert got == (v["ret"], v["err"]), v["name"]
            st = Stats()
            eng.bcc_last_batch_stats(ctypes.byref(st))
            assert st.host_rounds == st.rounds
    finally:
        eng.bcc_set_host_small_round(0)


def test_set_devices_rejects_without_side_effect(eng):
    """A rejected bcc_set_devices call (negative id anywhere) leaves the device list unchanged."""
    engine_stub.set_devices(eng, [3, 4])
    arr = (ctypes.c_int * 2)(0, -1)
    assert eng.bcc_set_devices(arr, 2) == -1
    out = (ctypes.c_int * 8)()
    n = eng.bcc_get_devices(out, 8)
    assert list(out)[:n] == [3, 4]
    engine_stub.set_devices(eng, [])


def test_single_call_with_device_failure_verified_on_host():
    """Default policy: the single-item ABI returns the exact verdict after device failures."""
    import sys
    code = f"""
import ctypes, json, os, sys
sys.path.insert(0, {HERE!r})
from fixtures import load_json
L = ctypes.CDLL({SO!r})
for v in load_json("crate_vectors.json"):
    spk, tx = bytes.fromhex(v["spk"]), bytes.fromhex(v["tx"])
    L.bcc_debug_fail_device_rounds(2)
    e = ctypes.c_int(-1)
    r = L.bitcoinconsensus_verify_script_with_amount(spk, len(spk), ctypes.c_int64(v["amount"]),
                                                     tx, len(tx), v["nin"], v["flags"], ctypes.byref(e))
    assert (r, e.value) == (v["ret"], v["err"]), v["name"]
print("ok")
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok" in p.stdout, (p.returncode, p.stdout, p.stderr)


def test_single_call_aborts_without_verdict():
    """Under BCC_DEVICE_FAILURE=error the single-item ABI has no 'no verdict' code: after the
    device fails it aborts (libsecp256k1's illegal-argument behaviour) rather than report a valid
    spend as invalid."""
    import signal
    import sys
    code = f"""
import ctypes, json, os, sys
sys.path.insert(0, {HERE!r})
from fixtures import load_json
L = ctypes.CDLL({SO!r})
v = load_json("crate_vectors.json")[0]
spk, tx = bytes.fromhex(v["spk"]), bytes.fromhex(v["tx"])
L.bcc_debug_fail_device_rounds(2)
e = ctypes.c_int(-1)
r = L.bitcoinconsensus_verify_script_with_amount(spk, len(spk), ctypes.c_int64(v["amount"]), tx,
                                                 len(tx), v["nin"], v["flags"], ctypes.byref(e))
print("returned", r, e.value)
"""
    env = dict(os.environ, BCC_DEVICE_FAILURE="error")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env=env)
    assert p.returncode == -signal.SIGABRT, (p.returncode, p.stdout, p.stderr)
    assert "GPU unavailable" in p.stderr


def test_witness_without_p2sh_pinned(eng):
    """Documented divergence: WITNESS without P2SH.  The reference
    asserts (interpreter.cpp:2049) and aborts when such a witness spend succeeds; this engine
    evaluates it as if the assert were absent.  Pin the chosen behaviour for the crate's
    P2SH-P2WPKH and P2WSH vectors."""
    for v in load_json("crate_vectors.json"):
        if v["flags"] != 0xE15 or v["ret"] != 1:
            continue
        flags = 0xE15 & ~1  # VERIFY_ALL minus P2SH
        got = call(eng, bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"], flags)
        assert got[1] == 0, v["name"]
        # native P2WPKH / P2WSH spends do not need P2SH; a P2SH-wrapped witness spend without
        # P2SH evaluation is a plain P2SH hash check that the witness-bearing input then fails
        # with WITNESS_UNEXPECTED (the reference would assert here only on success)
        if v["name"].startswith("p2sh"):
            assert got[0] == 0, v["name"]


def test_multi_device_verify_batch_identical(eng):
    """Node sharding (§8e): verify_batch over 3 'devices' (the stub's pipeline ignores the id, but
    the grouping, the per-device worker threads and the verdict gather are the product's) equals
    the single-device results on every script case; the rounds really were split."""
    import engine_stub
    allc = cases()
    by_flags = {}
    for c in allc:
        by_flags.setdefault(c["flags"], []).append(c)
    cs = max(by_flags.values(), key=len)
    vs = [dict(spk=c["spk"], tx=c["tx"], amount=c["amount"], nin=c["nin"], flags=c["flags"]) for c in cs]
    rc1, single = _batch(eng, vs)
    try:
        engine_stub.set_devices(eng, [0, 1, 2])
        rc3, multi = _batch(eng, vs)
        st = Stats()
        eng.bcc_last_batch_stats(ctypes.byref(st))
    finally:
        engine_stub.set_devices(eng, [])
    assert multi == single and rc3 == rc1
    assert multi == [(c["ret"], c["err"]) for c in cs]
    assert st.devices == 3


def test_pubkey_verify_batch_sharded(eng):
    """bcc_pubkey_verify_batch(device = -1) over 3 devices: contiguous ranges, same verdicts."""
    import engine_stub
    from fixtures import ecdsa_tuples
    ts = ecdsa_tuples() * 6
    one = engine_stub.pubkey_verify(eng, ts, 0)
    try:
        engine_stub.set_devices(eng, [0, 1, 2])
        many = engine_stub.pubkey_verify(eng, ts, -1)
    finally:
        engine_stub.set_devices(eng, [])
    assert many == one
    assert list(one) == [t["verdict"] for t in ts]


def _many_input_legacy_tx(R, O, n_in, seed):
    """A version-1 tx with n_in P2PKH inputs signed SIGHASH_ALL by the reference; returns
    (tx bytes, [spk per input])."""
    import hashlib
    import random
    from script_asm import hash160
    rng = random.Random(seed)

    def ser_var(n):
        return bytes([n]) if n < 253 else b"\xfd" + n.to_bytes(2, "little")

    def push(b):
        return (bytes([len(b)]) if len(b) < 76 else b"\x4c" + bytes([len(b)])) + b

    keys, spks = [], []
    for i in range(n_in):
        sk = hashlib.sha256(b"tplmid%d-%d" % (seed, i)).digest()
        pub = R.pubkey_create(sk, compressed=(i % 3 != 0))
        h = hash160(pub)
        keys.append((sk, pub))
        spks.append(b"\x76\xa9\x14" + h + b"\x88\xac")
    prev = [rng.randbytes(32) + rng.getrandbits(8).to_bytes(4, "little") for _ in range(n_in)]
    outs = b"".join((1000 + k).to_bytes(8, "little") + push(b"\x76\xa9\x14" + rng.randbytes(20) + b"\x88\xac")
                    for k in range(2))

    def ser(script_sigs):
        v = (1).to_bytes(4, "little") + ser_var(n_in)
        for i in range(n_in):
            v += prev[i] + ser_var(len(script_sigs[i])) + script_sigs[i] + b"\xff\xff\xff\xff"
        return v + ser_var(2) + outs + (0).to_bytes(4, "little")

    unsigned = ser([b""] * n_in)
    sigs = []
    for i in range(n_in):
        m = O.sighash(unsigned, i, spks[i], 1, 0, 0)
        sigs.append(push(R.sign(keys[i][0], m) + b"\x01") + push(keys[i][1]))
    return ser(sigs), spks


@pytest.mark.parametrize("chain_blocks,early,devs", [(0, 1, []), (1, 1, []), (12, 0, []), (160, 1, []),
                                                     (160, 0, []), (1, 1, [0, 1, 2]), (12, 1, [0, 0])])
def test_many_input_legacy_tx_template_midstates(eng, chain_blocks, early, devs):
    """Legacy txs of 12..250 P2PKH inputs (templates of 8..160 blocks: every job carries the
    template midstates, TPL_MID) through verify_batch: the stub evaluates each template job from
    the full preimage with the oracle and aborts if the product's midstate path disagrees; jobs
    whose remaining blocks exceed chain_blocks are hashed on the host from their midstate.  All
    inputs valid, and a byte flipped in the 40-input tx's first inputs or the 90-input tx's first
    outpoint gives the reference's (ret, err) for every input.  early: the P2PKH (key, signature)
    pairs are pre-extracted (bcc_set_early_q) and every deferred row is mapped to its early twin,
    which the stub checks byte for byte (engine_host_stub.cpp check_early_twins), and with it the
    early sighash of every long-template job (check_early_msgs).  devs: a
    multi-device list (no early rows there), whose device workers all wait for the one host pass
    over the offloaded chains (LateHost) before their G ladders."""
    from oracle_ctypes import Oracle, Reference, reference_available
    if not reference_available():
        pytest.skip("oracle/_ref not built")
    R, O = Reference(), Oracle()
    eng.bcc_set_host_chain_blocks.argtypes = [ctypes.c_uint]
    # 250 inputs: a 160-block template, whose first inputs' chains (>= 96 blocks from their
    # midstate) get early sighashes
    txs = [_many_input_legacy_tx(R, O, n, 11 + n) for n in (12, 40, 90, 250)]
    # mutations: byte 200 of the 40-input tx (its first inputs), an outpoint byte of input 0
    tx40 = bytearray(txs[1][0])
    tx40[200] ^= 0x01
    tx90 = bytearray(txs[2][0])
    tx90[5 + 3] ^= 0x10
    txs = txs[:3] + [(bytes(tx40), txs[1][1]), (bytes(tx90), txs[2][1])] + txs[3:]
    items, keep, exp = [], [], []
    for tx, spks in txs:
        bt = ctypes.create_string_buffer(tx, len(tx))
        keep.append(bt)
        for i, spk in enumerate(spks):
            bs = ctypes.create_string_buffer(spk, len(spk))
            keep.append(bs)
            items.append(Item(ctypes.addressof(bs), len(spk), 0, ctypes.addressof(bt), len(tx), i))
            exp.append(R.verify_script_with_amount(spk, 0, tx, i, 0x805))
    arr = (Item * len(items))(*items)
    ret = (ctypes.c_int * len(arr))()
    err = (ctypes.c_int * len(arr))()
    eng.bcc_set_early_q.argtypes = [ctypes.c_int]
    eng.stub_early_checked.restype = ctypes.c_size_t
    eng.stub_early_msg_checked.restype = ctypes.c_size_t
    checked0 = eng.stub_early_checked()
    msg0 = eng.stub_early_msg_checked()
    try:
        eng.bcc_set_host_chain_blocks(chain_blocks)
        eng.bcc_set_early_q(early)
        engine_stub.set_devices(eng, devs)
        eng.bitcoinconsensus_verify_batch(arr, len(arr), 0x805, ret, err)
        st = Stats()
        eng.bcc_last_batch_stats(ctypes.byref(st))
    finally:
        engine_stub.set_devices(eng, [])
        eng.bcc_set_host_chain_blocks(HOST_CHAIN_BLOCKS_DEFAULT)
        eng.bcc_set_early_q(1)
    assert list(zip(ret, err)) == exp
    if chain_blocks in (1, 12):
        assert st.host_hashed > 0
    if len(devs) > 1:
        assert st.devices == len(devs) and st.early_rows == 0
    elif early:
        # every input is a P2PKH spend with one check: one early row each, and the first round's
        # rows (the only round) all mapped to their twins; every device template job (all of them
        # unless chain_blocks sends long ones to the host) takes its twin's early sighash, which the
        # stub compares with the job's own digest
        assert st.early_rows == len(items) and st.early_mapped == len(items)
        assert eng.stub_early_checked() - checked0 == len(items)
        assert eng.stub_early_msg_checked() - msg0 == st.early_msgs
        if chain_blocks in (0, 160):
            assert st.early_msgs > 0  # the 250-input tx's long chains
        else:
            assert st.early_msgs < len(items)  # the long remainders went to the host
    else:
        assert st.early_rows == 0 and st.early_mapped == 0
    # the originals all valid; both flips sit in bytes every legacy preimage of their tx contains
    assert sum(r for r, _ in exp) == 12 + 40 + 90 + 250
