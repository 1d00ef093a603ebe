"""GPU parity of config C3 (block replay through bitcoinconsensus_verify_batch): transactions of
the reference benchmark block's shape (tests/golden/block413567_shape.json), mixed P2PKH /
P2WPKH / P2SH 2-of-3 multisig inputs, verified end to end (threaded host interpreter + GPU
sighash + GPU ECDSA, re-run rounds for CHECKMULTISIG key advance) and compared item by item with
the reference library (oracle/_ref) on the same bytes, unmutated and mutated."""
import json
import os
import random

import pytest

from oracle_ctypes import Reference, reference_available

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def block_shape():
    return [tuple(t) for t in json.load(open(os.path.join(HERE, "golden", "block413567_shape.json")))["txs"]]


@pytest.fixture(scope="module")
def wl():
    import bitcoinconsensus_amd as B
    sh = block_shape()
    big = max(sh, key=lambda t: t[0])
    sub = sh[:160] + [big] + sh[-40:]
    return B.Workload(kind="block", shape=sub, seed=0x5EED0003)


@pytest.mark.parametrize("chain_blocks,bip143_blocks", [(32, 32), (0, 32), (0, 0)])
def test_block_workload_all_valid_and_matches_reference(wl, chain_blocks, bip143_blocks):
    """chain_blocks 32: the big txs' long legacy chains hashed on the host (during the device
    round); bip143_blocks 32 (default): their BIP143 per-tx digests and preimages on the host;
    (0, 0): every chain in a GPU lane."""
    import bitcoinconsensus_amd as B
    B.set_host_chain_blocks(chain_blocks)
    B.set_host_bip143_blocks(bip143_blocks)
    try:
        n_valid, ret = wl.verify_batch()
        st = B.last_batch_stats()
    finally:
        B.set_host_chain_blocks(B.HOST_CHAIN_BLOCKS_DEFAULT)
        B.set_host_bip143_blocks(32)
    assert (st["host_hashed"] > 0) == (chain_blocks + bip143_blocks > 0)
    assert n_valid == wl.n and all(r == 1 for r in ret)
    assert st["rounds"] == 1          # multisig candidate pairs are queued up front: no re-run
    assert st["tuples"] > wl.n        # multisig inputs verify 2-3 signatures
    if reference_available():
        R = Reference()
        for i in range(wl.n):
            spk, amt, tx, nin = wl.item(i)
            assert R.verify_script_with_amount(spk, amt, tx, nin, B.VERIFY_ALL) == (1, 0), i


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("chain_blocks", [0, 16])
def test_block_workload_mutations_match_reference(wl, chain_blocks):
    """Single-byte flips anywhere in a spending transaction (signatures, pubkeys, scripts,
    outpoints, amounts, lengths) under three flag sets: per-item (ret, err) equals the reference.
    chain_blocks 16: the many-input txs' chains hashed on the host while the device round runs
    (their digests reach the message rows before the G ladder)."""
    import bitcoinconsensus_amd as B
    B.set_host_chain_blocks(chain_blocks)
    try:
        _mutations(B, wl)
        if chain_blocks:
            assert B.last_batch_stats()["host_hashed"] > 0
    finally:
        B.set_host_chain_blocks(B.HOST_CHAIN_BLOCKS_DEFAULT)


def _mutations(B, wl):
    R = Reference()
    rng = random.Random(3)
    items = []
    for _ in range(300):
        spk, amt, tx, nin = wl.item(rng.randrange(wl.n))
        tx = bytearray(tx)
        for _ in range(rng.choice((0, 1, 1, 2))):
            tx[rng.randrange(len(tx))] ^= 1 << rng.randrange(8)
        if rng.random() < 0.1:
            amt += 1
        items.append((spk, amt, bytes(tx), nin))
    for flags in (B.VERIFY_ALL, B.VERIFY_P2SH | B.VERIFY_DERSIG, B.VERIFY_NONE):
        got = [(r, int(e)) for r, e in B.verify_batch(items, flags)]
        exp = [R.verify_script_with_amount(s, a, t, k, flags) for s, a, t, k in items]
        assert got == exp


def test_block_workload_device_fault_with_early_work(wl):
    """Round 5: the block call runs early Q halves and early sighashes (flagged TPL_EARLY jobs whose
    digests the round copies from the early set).  One injected device fault: the round is retried
    on a fresh device batch, which has no early state, so staging must clear the flags and hash
    those jobs itself; every input stays valid, as the reference says.  (The host fallback, which
    hashes flagged jobs like any other, is covered on the CPU: test_host_engine.py's failure tests
    run with early work on; here the autouse fixture forbids host rounds.)"""
    faults = 1
    import bitcoinconsensus_amd as B
    B.set_host_chain_blocks(B.HOST_CHAIN_BLOCKS_DEFAULT)
    n_valid, _ = wl.verify_batch()
    st = B.last_batch_stats()
    assert n_valid == wl.n
    assert st["early_rows"] > 0 and st["early_msgs"] > 0  # the paths under test are in use
    B.debug_fail_device_rounds(faults)
    try:
        n_valid, ret = wl.verify_batch()
        st = B.last_batch_stats()
    finally:
        B.debug_fail_device_rounds(0)
    assert n_valid == wl.n and all(r == 1 for r in ret)
    assert st["device_retries"] >= 1 and st["host_rounds"] == 0


@pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")
def test_full_c3_block_matches_reference():
    """C3 at the bench's full size (bench.py DEFAULT_N: 4,000 txs with block413567's histogram
    tiled, 13,170 inputs, seed 0x5EED0003): one bitcoinconsensus_verify_batch call with the
    default host/device split, every item's (ret, err) against the reference's
    bitcoinconsensus_verify_script_with_amount on the same bytes, unmutated.  Then a second batch
    with ~3 % of the items mutated (single bit flips, amount changes), again item by item."""
    import bitcoinconsensus_amd as B
    sh = block_shape()
    txs = (sh * (4000 // len(sh) + 1))[:4000]
    w = B.Workload(kind="block", shape=txs, seed=0x5EED0003)
    try:
        assert w.n == 13170
        items = [w.item(i) for i in range(w.n)]
        R = Reference()
        ref, _ = R.bulk_verify_script(items, B.VERIFY_ALL)
        assert all(r == (1, 0) for r in ref)
        rc, got = B.verify_batch_raw(items)
        assert rc == w.n and got == ref
        st = B.last_batch_stats()
        assert st["host_rounds"] == 0 and st["tuples"] > w.n
        rng = random.Random(0xC3)
        mut = []
        for spk, amt, tx, nin in items:
            if rng.random() < 0.03:
                tx = bytearray(tx)
                if rng.random() < 0.8:
                    k = rng.randrange(len(tx))
                    tx[k] ^= 1 << rng.randrange(8)
                else:
                    amt += rng.choice((-1, 1))
                tx = bytes(tx)
            mut.append((spk, amt, tx, nin))
        ref, _ = R.bulk_verify_script(mut, B.VERIFY_ALL)
        rc, got = B.verify_batch_raw(mut)
        bad = [i for i in range(len(mut)) if got[i] != ref[i]]
        assert not bad, [(i, got[i], ref[i]) for i in bad[:10]]
        assert rc == sum(r for r, _ in ref) and rc < w.n
    finally:
        w.free()


def test_block_workload_rows_exceed_items_bench_abi(wl):
    """The bench library's row accessors on a block workload whose 2-of-3 multisig inputs stage
    several tuple rows each (the round-5 abort: an item-sized verdict buffer): verdicts(),
    msgs() and tuple_items() are sized by rows, and each C entry point refuses a buffer one row
    short with BCC_BENCH_ERR_CAPACITY (-2) instead of writing past it."""
    import ctypes
    import bitcoinconsensus_amd as B
    w = B.Workload(kind="block", shape=block_shape()[:60], seed=0x5EED0013)
    try:
        t = w.shape()["tuples"]
        assert t > w.n
        w.run()
        v = w.verdicts()
        # (2-of-3 candidate pairs: some rows pair a signature with the wrong key -> 0)
        assert len(v) == t and set(v) <= {0, 1} and sum(v) >= w.n
        ti = w.tuple_items()
        assert len(ti) == t and max(ti) < w.n and sorted(set(ti)) == list(range(w.n))
        m = w.msgs()
        assert len(m) == 32 * t and m.count(bytes(32)) == 0
        L = B.blib()
        short = ctypes.create_string_buffer(t + 64)
        assert L.bcc_workload_verdicts(w.h, short, t - 1) == -2
        assert short.raw[:t] == bytes(t)  # nothing written
        assert L.bcc_workload_msgs(w.h, short, 32 * t - 1) == -2
        u = (ctypes.c_uint32 * t)()
        assert L.bcc_workload_tuple_items(w.h, u, t - 1) == -2
        assert L.bcc_workload_verdicts(w.h, short, t) == 0 and short.raw[:t] == v
        assert L.bcc_workload_verdicts(None, short, t) == -1
    finally:
        w.free()
