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
