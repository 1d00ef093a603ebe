"""GPU parity of both signature paths in one run: the default square-root-free path (every other
GPU test) and the round-1 path kept behind BCC_ECDSA_PATH=legacy (read once per process, so it runs
in one child process): the reference-labelled ECDSA tuple fixtures and BIP340 vectors / tuples
through the C ABI, and identical verdicts from both paths on a mutated random sample."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = r'''
import json, random, sys
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import bitcoinconsensus_amd as B
from fixtures import bip340_vectors, ecdsa_tuples, pub_to_tuple, schnorr_tuples
from oracle_ctypes import Oracle
O = Oracle()
ts = ecdsa_tuples()
rng = random.Random(77)
for i in range(2000):  # mutated copies of valid tuples
    t = dict(rng.choice([t for t in ts[:500] if t["verdict"] == 1]))
    h = bytearray(t["hash"]); h[rng.randrange(32)] ^= (i & 1) << rng.randrange(8); t["hash"] = bytes(h)
    ts.append(t)
pub65, msg, r32, s32 = bytearray(), bytearray(), bytearray(), bytearray()
for t in ts:
    tag, x, y = pub_to_tuple(t["pub"])
    ok, r, s = O.der_parse_lax(t["sig"])
    if not ok:
        r = s = bytes(32)
    pub65 += bytes([tag]) + x + y; msg += t["hash"]; r32 += r; s32 += s
ev = list(B.ecdsa_verify_tuples(bytes(pub65), bytes(msg), bytes(r32), bytes(s32), 0))
ss = bip340_vectors() + schnorr_tuples()
sv = list(B.schnorr_verify_tuples(b"".join(t["sig"] for t in ss), b"".join(t["msg"] for t in ss),
                                  b"".join(t["pub"] for t in ss), 0))
print(json.dumps({"ecdsa": ev, "schnorr": sv, "n_fixture": len(ecdsa_tuples())}))
'''


def _run(path):
    env = dict(os.environ)
    env.pop("BCC_ECDSA_PATH", None)
    if path:
        env["BCC_ECDSA_PATH"] = path
    out = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "rust-bitcoinconsensus_amd"),
                          HERE], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_legacy_and_twist_paths_agree_with_reference():
    from fixtures import bip340_vectors, ecdsa_tuples, schnorr_tuples
    ref_e = [t["verdict"] for t in ecdsa_tuples()]
    ref_s = [t["verdict"] for t in bip340_vectors() + schnorr_tuples()]
    legacy, twist = _run("legacy"), _run(None)
    n = legacy["n_fixture"]
    for got in (legacy, twist):
        assert got["ecdsa"][:n] == ref_e
        assert got["schnorr"] == ref_s
    assert legacy["ecdsa"] == twist["ecdsa"]  # the mutated sample too
