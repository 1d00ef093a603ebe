"""CPU: the kernel's per-lane arithmetic (csrc/ecdsa_lane.h, compiled for the host by
tests/native/lane_host.cpp -- test-only, never part of the product) against the reference
fixtures. Lets the exact lane code be checked without a GPU."""
import ctypes
import os
import subprocess

import pytest

from fixtures import ecdsa_tuples, pub_to_tuple
from oracle_ctypes import Oracle

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "_build", "lane_host.so")


@pytest.fixture(scope="module")
def lane():
    src = os.path.join(HERE, "native", "lane_host.cpp")
    deps = [src] + [os.path.join(HERE, "..", "rust-bitcoinconsensus_amd", "csrc", f)
                    for f in ("ecdsa_lane.h", "secp256k1_device.h")]
    if not os.path.exists(SO) or any(os.path.getmtime(d) > os.path.getmtime(SO) for d in deps):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO, src])
    return ctypes.CDLL(SO)


def test_lane_code_matches_reference_fixtures(lane):
    O = Oracle()
    ts = ecdsa_tuples()
    bad = []
    for i, t in enumerate(ts[::3]):  # every 3rd tuple keeps the CPU run short
        tag, x, y = pub_to_tuple(t["pub"])
        ok, r, s = O.der_parse_lax(t["sig"])
        if not ok:
            r = s = bytes(32)
        got = lane.lane_verify(tag, x, y, r, s, t["hash"])
        if got != t["verdict"]:
            bad.append((t["cls"], got, t["verdict"]))
    assert not bad, bad[:10]
