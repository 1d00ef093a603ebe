"""CPU: the engine's host verification (csrc/host/host_verify.cpp: the kernels' lane code compiled
for the CPU, the engine's own sighash job evaluation), which the library uses for device-failure
fallback and small rounds, against the REFERENCE's verdicts:

* bcc_host_verify_tuples over every committed adversarial tuple class (tests/golden/
  ecdsa_tuples.npz, verdicts from CPubKey::Verify, pubkey.cpp:191-207);
* host_sighash over the reference's sighash goldens (through test_sighash_goldens' checks) is
  covered by test_host_engine.py's fallback tests (every script-level golden, every device round
  verified on the host).

Built into tests/native/_build/engine_host.so with the rest of csrc/host (test build); the same
source is compiled into librbc_amd.so."""
import ctypes

from engine_stub import load
from fixtures import ecdsa_tuples, pub_to_tuple
from oracle_ctypes import Oracle


def test_host_verify_tuples_match_reference_fixtures():
    L = load()
    L.bcc_host_verify_tuples.argtypes = [ctypes.c_char_p] * 4 + [ctypes.c_char_p, ctypes.c_size_t,
                                                                 ctypes.c_uint]
    O = Oracle()
    ts = ecdsa_tuples()
    pub, msg, r32, s32 = bytearray(), bytearray(), bytearray(), bytearray()
    for t in ts:
        tag, x, y = pub_to_tuple(t["pub"])
        ok, r, s = O.der_parse_lax(t["sig"])
        if not ok:
            r = s = bytes(32)
        pub += bytes([tag]) + x + y
        msg += t["hash"]
        r32 += r
        s32 += s
    out = ctypes.create_string_buffer(len(ts))
    assert L.bcc_host_verify_tuples(bytes(pub), bytes(msg), bytes(r32), bytes(s32), out, len(ts),
                                    4) == 0
    bad = [(t["cls"], i) for i, t in enumerate(ts) if out.raw[i] != t["verdict"]]
    assert not bad, bad[:10]
    assert len({t["cls"] for t in ts}) >= 15 and sum(t["verdict"] for t in ts) > 500
