"""CPU: the interpreter's small-block allocator (csrc/host/pool.cpp) -- content integrity under
many short-lived threads (the engine spawns its host threads per call) and bounded growth: blocks
freed by exited threads return to the reservoir and are reused."""
import ctypes
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "_build", "pool_test.so")


@pytest.fixture(scope="module")
def pool():
    src = os.path.join(HERE, "native", "pool_test.cpp")
    lib = os.path.join(HERE, "..", "rust-bitcoinconsensus_amd", "csrc", "host", "pool.cpp")
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-o", SO,
                           src, lib])
    L = ctypes.CDLL(SO)
    L.pool_stress.restype = ctypes.c_long
    L.pool_chunk_count.restype = ctypes.c_size_t
    return L


def test_pool_content_and_bounded_growth(pool):
    assert pool.pool_stress(8, 20000, 1) == 0
    after_first = pool.pool_chunk_count()
    for r in range(2, 8):  # fresh threads every round, same workload shape
        assert pool.pool_stress(8, 20000, r) == 0
    # the later rounds reuse the reservoir: growth stays within a small factor of one round's peak
    assert pool.pool_chunk_count() <= 3 * after_first + 8
