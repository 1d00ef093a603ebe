"""GPU: node sharding inside the library on the hardware at hand.  The device list
names device 0 twice, so two persistent worker threads with their own streams, device batches and
scratch drive the same MI355X concurrently through exactly the code that spreads a round over
several GPUs; results must be identical to the single-device engine and to the reference."""
import pytest

from oracle_ctypes import reference_available

pytestmark = pytest.mark.gpu


@pytest.fixture()
def two_workers():
    import bitcoinconsensus_amd as B
    B.set_devices([0, 0])
    yield B
    B.set_devices([])


def test_block_workload_sharded_equals_single(two_workers):
    B = two_workers
    import json
    import os
    shape = [tuple(t) for t in json.load(open(os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "golden", "block413567_shape.json")))["txs"]]
    B.set_devices([])
    wl = B.Workload(kind="block", shape=shape[:400], seed=0x5EED0003)
    items = [wl.item(i) for i in range(wl.n)]
    single = B.verify_batch(items)
    B.set_devices([0, 0])
    multi = B.verify_batch(items)
    st = B.last_batch_stats()
    assert multi == single
    assert all(r == 1 for r, _ in multi)
    assert st["devices"] == 2
    # mutated: the sharded engine still matches the reference item by item
    if reference_available():
        import random
        from oracle_ctypes import Reference
        R = Reference()
        rng = random.Random(7)
        mut = []
        for spk, amt, tx, nin in items[:2000]:
            tx = bytearray(tx)
            if rng.random() < 0.3:
                tx[rng.randrange(len(tx))] ^= 1 << rng.randrange(8)
            mut.append((spk, amt, bytes(tx), nin))
        got = [(r, int(e)) for r, e in B.verify_batch(mut)]
        exp, _ = R.bulk_verify_script(mut, B.VERIFY_ALL)
        assert got == exp


def test_pubkey_verify_batch_sharded(two_workers):
    B = two_workers
    from fixtures import ecdsa_tuples
    ts = ecdsa_tuples() * 8
    tuples = [(t["pub"], t["hash"], t["sig"]) for t in ts]
    many = B.pubkey_verify_batch(tuples, device=-1)
    one = B.pubkey_verify_batch(tuples, device=0)
    assert many == one
    assert list(one) == [t["verdict"] for t in ts]


def test_rank_partition_of_one_global_set():
    """bench.py's multi-GPU partition: rank r stages items [r n, (r + 1) n) of ONE
    global set (Workload(n, first=r n), TupleSet(n, first=r n, total=N n)).  Two ranges must be
    exactly the items, sighashes and verdicts of the single 2n set -- no overlap, no gap, no
    rank-dependent content."""
    import bitcoinconsensus_amd as B
    n, seed = 2500, 0x5EED0001
    full = B.Workload(2 * n, seed=seed)
    parts = [B.Workload(n, seed=seed, first=0), B.Workload(n, seed=seed, first=n)]
    assert [full.item(i) for i in range(2 * n)] == [p.item(i) for p in parts for i in range(n)]
    full.run()
    for p in parts:
        p.run()
    assert full.msgs() == b"".join(p.msgs() for p in parts)
    assert full.verdicts() == b"".join(p.verdicts() for p in parts)
    assert all(full.verdicts())
    # the C4 tuple sets the same way (10 % adversarial classes drawn per global row)
    t_full = B.TupleSet(2 * n, kind="c4")
    t_parts = [B.TupleSet(n, kind="c4", first=0, total=2 * n),
               B.TupleSet(n, kind="c4", first=n, total=2 * n)]
    hf = t_full.host()
    hp = [t.host() for t in t_parts]
    assert bytes(hf["msg32"]) == b"".join(bytes(h["msg32"]) for h in hp)
    assert bytes(hf["cls"]) == b"".join(bytes(h["cls"]) for h in hp)
    for t in [t_full] + t_parts:
        t.run()
    assert t_full.verdicts() == b"".join(t.verdicts() for t in t_parts)
    assert t_full.verdicts() == bytes(hf["expect"])


def test_eight_entry_device_list():
    """The node shape: an 8-entry device list, here device 0 eight times, so eight
    persistent per-GPU workers with their own streams, arenas and scratch split each round of
    verify_batch (cut at transaction boundaries) and each tuple batch (equal ranges) -- the same
    code path an 8 x MI355X node runs.  Verdicts equal the single-device engine's and the
    reference labels."""
    import json
    import os
    import bitcoinconsensus_amd as B
    from fixtures import ecdsa_tuples
    shape = [tuple(t) for t in json.load(open(os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "golden", "block413567_shape.json")))["txs"]]
    wl = B.Workload(kind="block", shape=shape[:800], seed=0x5EED0013)
    items = [wl.item(i) for i in range(wl.n)]
    ts = ecdsa_tuples() * 16
    tuples = [(t["pub"], t["hash"], t["sig"]) for t in ts]
    B.set_devices([])
    single = B.verify_batch(items)
    one = B.pubkey_verify_batch(tuples, device=0)
    try:
        B.set_devices([0] * 8)
        assert B.get_devices() == [0] * 8
        multi = B.verify_batch(items)
        st = B.last_batch_stats()
        many = B.pubkey_verify_batch(tuples, device=-1)
    finally:
        B.set_devices([])
    assert st["devices"] == 8
    assert multi == single and all(r == 1 for r, _ in multi)
    assert many == one and list(one) == [t["verdict"] for t in ts]


def test_sharded_round_with_host_chains(two_workers):
    """Round 5: multi-device rounds offload long legacy chains too (LateHost).  Device list [0, 0]
    over the block shape's largest tx among ordinary ones, chains above 16 blocks hashed on the host
    while both workers' device batches run their message-independent kernels (each worker's round
    waits for the one host pass): host_hashed > 0, two devices used, verdicts equal to the
    single-device run, and (mutated) equal to the reference item by item."""
    B = two_workers
    import json
    import os
    import random
    shape = [tuple(t) for t in json.load(open(os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "golden", "block413567_shape.json")))["txs"]]
    big = max(shape, key=lambda t: t[0])
    wl = B.Workload(kind="block", shape=shape[:120] + [big] + shape[-60:], seed=0x5EED0023)
    items = [wl.item(i) for i in range(wl.n)]
    rng = random.Random(11)
    mut = []
    for spk, amt, tx, nin in items:
        tx = bytearray(tx)
        if rng.random() < 0.2:
            tx[rng.randrange(len(tx))] ^= 1 << rng.randrange(8)
        mut.append((spk, amt, bytes(tx), nin))
    B.set_host_chain_blocks(16)
    try:
        B.set_devices([])
        single = B.verify_batch(items)
        single_mut = B.verify_batch(mut)
        B.set_devices([0, 0])
        multi = B.verify_batch(items)
        st = B.last_batch_stats()
        multi_mut = B.verify_batch(mut)
        st_mut = B.last_batch_stats()
    finally:
        B.set_host_chain_blocks(B.HOST_CHAIN_BLOCKS_DEFAULT)
    assert st["devices"] == 2 and st["host_hashed"] > 0 and st_mut["host_hashed"] > 0
    assert multi == single and all(r == 1 for r, _ in multi)
    assert multi_mut == single_mut
    if reference_available():
        from oracle_ctypes import Reference
        exp, _ = Reference().bulk_verify_script(mut, B.VERIFY_ALL)
        assert [(r, int(e)) for r, e in multi_mut] == exp
