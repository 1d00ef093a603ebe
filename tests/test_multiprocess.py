"""CPU, world_size 2 and 4 over gloo: the multi-GPU bench path's aggregation (max wall time over
ranks, sum of valid verdicts) and per-rank shard seeding, exercised without a GPU."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    elapsed, valid = bench.aggregate(1.0 + rank, 100 + rank, world, device="cpu")
    q.put((rank, elapsed, valid))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_aggregate_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    want_t = float(world)  # max over ranks of 1 + rank
    want_v = sum(100 + r for r in range(world))
    assert res == [(r, want_t, want_v) for r in range(world)]


def _shard_worker(rank, world, port, q):
    """One rank of a sharded C4-style run: verdicts for its contiguous range of ONE global tuple
    set (the product's host front end + the oracle-stubbed device pipeline), then bench.py's
    bitmap all-gather."""
    import torch.distributed as dist
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import engine_stub
    from fixtures import ecdsa_tuples
    ts = ecdsa_tuples() * 3
    n = len(ts)
    lo, hi = n * rank // world, n * (rank + 1) // world
    L = engine_stub.load()
    local = engine_stub.pubkey_verify(L, ts[lo:hi])
    full = bench.gather_verdicts(list(local), world, device="cpu")
    q.put((rank, bytes(full.tolist())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_tuple_set_gather_gloo(world):
    """§8e: `world` ranks each verify their contiguous range of one tuple set; the gathered validity
    bitmap equals the single-process verdicts (and the reference's labels)."""
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    import engine_stub
    from fixtures import ecdsa_tuples
    engine_stub.load()  # build once, before the ranks start
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
        assert p.exitcode == 0
    res = dict(q.get() for _ in range(world))
    ts = ecdsa_tuples() * 3
    single = engine_stub.pubkey_verify(engine_stub.load(), ts)
    assert all(res[r] == single for r in range(world))
    assert list(single) == [t["verdict"] for t in ts]


def test_single_rank_passthrough():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.aggregate(3.5, 7, 1) == (3.5, 7)
