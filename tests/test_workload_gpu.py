"""GPU parity of config C2 on the EXACT path bench.py times (BASELINE.json configs[1]).

bench.py's C2 step is Workload.run: the staged first-round batch (BIP143 sighash kernels + the
ECDSA kernels K_inv / K_key / K_prep / K_ladder) over synthetic P2WPKH spends resident in HBM.
These tests run that same staged path on the seed the bench uses, unmutated and with ~10 % of the
items mutated by single-byte flips (signature, pubkey, amount, witness / any tx byte), and
compare against the REFERENCE (oracle/_ref, Bitcoin Core v0.21 libbitcoinconsensus):

* tuple level: every staged tuple's sighash row and verdict against the (sighash, verdict) the
  reference's own interpreter produced for that item (ref_capture_script records
  GenericTransactionSignatureChecker::VerifyECDSASignature, interpreter.cpp:1644-1676);
* item level: bitcoinconsensus_verify_batch (ret, err) per item against
  bitcoinconsensus_verify_script_with_amount (bitcoinconsensus.cpp:104-110).
"""
import random

import pytest

from oracle_ctypes import Reference, reference_available

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built")]

# above one K_keyq residency round (256 CUs x 4 SIMDs x 4 waves x 64 = 262,144 lanes): the staged
# round runs the split K_keyq with the full round's G ladder beside the tail (round 6)
N = 300_000
SEED = 0x5EED0001  # bench.py SEEDS["c2"]


@pytest.fixture(scope="module")
def wl():
    import bitcoinconsensus_amd as B
    w = B.Workload(N, seed=SEED)
    yield w
    w.free()


def _witness_spans(tx):
    """(sig_start, sig_len, pub_start, pub_len) of a C2 tx (1-in / 1-out segwit, 2 witness items)."""
    # version 4 | marker flag 2 | vin count 1 | outpoint 36 | script len 1 | seq 4 | vout count 1
    o = 4 + 2 + 1 + 36 + 1 + 4
    nout = tx[o]
    o += 1
    for _ in range(nout):
        o += 8
        o += 1 + tx[o]
    assert tx[o] == 2
    o += 1
    sl = tx[o]
    sig = (o + 1, sl)
    o += 1 + sl
    pl = tx[o]
    return sig[0], sig[1], o + 1, pl


def mutate(rng, item):
    spk, amt, tx, nin = item
    tx = bytearray(tx)
    kind = rng.randrange(5)
    ss, sl, ps, pl = _witness_spans(tx)
    if kind == 0:            # signature byte (DER structure, r, s or the hashtype)
        tx[ss + rng.randrange(sl)] ^= 1 << rng.randrange(8)
    elif kind == 1:          # pubkey byte (header or x)
        tx[ps + rng.randrange(pl)] ^= 1 << rng.randrange(8)
    elif kind == 2:          # amount (BIP143 commits to it)
        amt += rng.choice((1, -1, 1 << 20))
    elif kind == 3:          # any other witness byte (lengths, item count)
        tx[ss - 2 + rng.randrange(3)] ^= 1 << rng.randrange(8)
    else:                    # any byte of the transaction
        tx[rng.randrange(len(tx))] ^= 1 << rng.randrange(8)
    return spk, amt, bytes(tx), nin, kind


def test_c2_staged_unmutated_matches_reference(wl):
    """All N staged verdicts are 1, tuples map 1:1 onto items, and the reference accepts every
    item; a sample's sighash rows equal the reference's own sighashes."""
    import bitcoinconsensus_amd as B
    wl.run()
    v = wl.verdicts()
    ti = wl.tuple_items()
    assert len(v) == N and ti == list(range(N))
    R = Reference()
    items = [wl.item(i) for i in range(N)]
    ref, _ = R.bulk_verify_script(items, B.VERIFY_ALL)
    mism = [i for i in range(N) if (ref[i][0] == 1) != (v[i] == 1)]
    assert not mism, mism[:10]
    assert all(r == (1, 0) for r in ref)
    msgs = wl.msgs()
    rng = random.Random(1)
    for i in rng.sample(range(N), 2000):
        r, _, recs = R.capture_script(*items[i], B.VERIFY_ALL)
        assert r == 1 and len(recs) == 1
        assert msgs[32 * i: 32 * i + 32] == recs[0]["sighash"], i


def test_c2_staged_mutated_matches_reference(wl):
    """~10 % of the C2 items mutated, staged through the same first-round path: every tuple's
    (sighash, verdict) equals the reference interpreter's, unmutated items stay valid, and
    verify_batch's per-item (ret, err) equals the reference on all N items."""
    import bitcoinconsensus_amd as B
    R = Reference()
    rng = random.Random(0xC2)
    items, kinds = [], {}
    for i in range(N):
        it = wl.item(i)
        if rng.random() < 0.10:
            spk, amt, tx, nin, k = mutate(rng, it)
            items.append((spk, amt, tx, nin))
            kinds[i] = k
        else:
            items.append(it)
    w = B.Workload(kind="items", items=items)
    try:
        w.run()
        v = w.verdicts()
        ti = w.tuple_items()
        msgs = w.msgs()
    finally:
        w.free()
    by_item = {}
    for t, i in enumerate(ti):
        by_item.setdefault(i, []).append((msgs[32 * t: 32 * t + 32], v[t]))
    # unmutated items: exactly one tuple, verified true
    for i in range(N):
        if i not in kinds:
            assert by_item.get(i) == [(by_item[i][0][0], 1)], i
    # mutated items: every GPU tuple is one of the reference's checks with the same verdict, and
    # every check the reference accepted was deferred to the GPU.  The one exception is the
    # device key-hash check (bcc_set_device_key_hash): a first run defers the signature check
    # with HASH160(key) == program attached, so an item whose key no longer hashes to its program
    # has a tuple the reference never reached (it stopped at OP_EQUALVERIFY, no checks): that
    # tuple's verdict must be 0.
    n_false = n_keyhash = 0
    for i in kinds:
        r, _, recs = R.capture_script(*items[i], B.VERIFY_ALL)
        gpu = by_item.get(i, [])
        ref_pairs = [(c["sighash"], c["verdict"]) for c in recs]
        for pair in gpu:
            if pair not in ref_pairs and not recs and r == 0 and pair[1] == 0:
                n_keyhash += 1
                continue
            assert pair in ref_pairs, (i, kinds[i])
            n_false += pair[1] == 0
        for pair in ref_pairs:
            if pair[1] == 1:
                assert pair in gpu, (i, kinds[i])
    assert n_false > 1000  # the mutations really exercise rejection on the GPU
    # item level, the drop-in
    got = [(r, int(e)) for r, e in B.verify_batch(items)]
    exp, _ = R.bulk_verify_script(items, B.VERIFY_ALL)
    bad = [i for i in range(N) if got[i] != exp[i]]
    assert not bad, [(i, kinds.get(i), got[i], exp[i]) for i in bad[:10]]
    assert sum(r for r, _ in exp) < N - len(kinds) // 2


def test_c2_mutated_drop_in_upload_modes_and_pipelined_chunks(wl):
    """The drop-in's host -> HBM paths give the reference's (ret, err) on every item: the direct
    upload from the host pass's page-locked arrays (default) and the pinned-image upload, each
    in one round and in pipelined chunks (chunk 64k: the caller stages every chunk's round while
    the worker runs the previous one, so the direct copies read arrays the next chunk must not
    touch)."""
    import bitcoinconsensus_amd as B
    R = Reference()
    rng = random.Random(0xD1)
    n = 200_000
    items = []
    for i in range(n):
        it = wl.item(i)
        items.append(mutate(rng, it)[:4] if rng.random() < 0.10 else it)
    exp, _ = R.bulk_verify_script(items, B.VERIFY_ALL)
    try:
        for chunk in (0, 64_000):
            B.set_pipeline_chunk(chunk)
            for direct in (True, False, True):
                B.set_direct_upload(direct)
                got = [(r, int(e)) for r, e in B.verify_batch(items)]
                bad = [i for i in range(n) if got[i] != exp[i]]
                assert not bad, (chunk, direct, [(i, got[i], exp[i]) for i in bad[:10]])
    finally:
        B.set_direct_upload(True)
        B.set_pipeline_chunk(500_000)


def test_c2_drop_in_concurrent_callers_direct_upload(wl):
    """Two threads calling the drop-in at once (ctypes drops the GIL), each on its own half of the
    300k C2 items with ~10 % mutated: first in one round each (150k rows: every large array goes
    up directly from the page-locked pool, so both threads' arrays are in flight together), then
    in pipelined 70k chunks (the raw txs direct, the rows through the image).  Every item's
    (ret, err) equals the reference's."""
    import threading
    import bitcoinconsensus_amd as B
    R = Reference()
    rng = random.Random(0xD2)
    items = []
    for i in range(N):
        it = wl.item(i)
        items.append(mutate(rng, it)[:4] if rng.random() < 0.10 else it)
    exp, _ = R.bulk_verify_script(items, B.VERIFY_ALL)
    errors = []

    def caller(k):
        mine = items[k::2]
        want = exp[k::2]
        for _ in range(2):
            got = [(r, int(e)) for r, e in B.verify_batch(mine)]
            bad = [i for i in range(len(mine)) if got[i] != want[i]]
            if bad:
                errors.append((k, bad[:5]))

    try:
        for chunk in (500_000, 70_000):
            B.set_pipeline_chunk(chunk)
            th = [threading.Thread(target=caller, args=(k,)) for k in range(2)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            assert not errors, (chunk, errors)
    finally:
        B.set_pipeline_chunk(500_000)
