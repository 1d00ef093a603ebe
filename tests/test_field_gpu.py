"""Device Fp arithmetic (csrc/fe_asm.h carry chains and their rare fold branches) against Python
integers.  Edge operands sit at lane positions mixed with random lanes, so waves that take the
wave-uniform rare branch also carry lanes that must come through it unchanged."""
import ctypes
import random

import pytest

P = 2**256 - 2**32 - 977
M256 = 2**256 - 1

EDGES = [0, 1, 2, 3, 976, 977, 978, 2**32 - 1, 2**32, 2**32 + 976, 2**32 + 977, 2**32 + 978,
         2**64 - 1, 2**224, 2**255 - 1, 2**255, 2**255 + 1, P - 2, P - 1, P, P + 1, P + 977,
         2**256 - 2**32 - 1, 2**256 - 2, 2**256 - 1, 2**256 - 2**33, (2**256 - 1) // 3]


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def pack(vals):
    arr = (ctypes.c_uint32 * (8 * len(vals)))()
    for i, v in enumerate(vals):
        for j, w in enumerate(limbs(v)):
            arr[8 * i + j] = w
    return arr


def unpack(arr, n):
    return [sum(arr[8 * i + j] << (32 * j) for j in range(8)) for i in range(n)]


def operand_pairs(seed=7, nrand=6000):
    rng = random.Random(seed)
    pairs = []
    for a in EDGES:
        for b in EDGES:
            pairs.append((a, b))
            # interleave random lanes between edge lanes
            pairs.append((rng.getrandbits(256), rng.getrandbits(256)))
    for _ in range(nrand):
        pairs.append((rng.getrandbits(256), rng.getrandbits(256)))
    for _ in range(500):  # both operands in [p, 2^256): double wrap-around territory
        pairs.append((P + rng.randrange(2**256 - P), P + rng.randrange(2**256 - P)))
    # limbs drawn from {0, 1, 2^32 - 1, 2^32 - 2, p's low limb, random}: products whose high
    # limbs sit at 2^32 - 1 take every rare carry of fe_reduce512_v4 (the D_k carries, the chain's
    # carry out of limb 8, the top fold's carries; about 15 % of these lanes in a Python model of
    # the reduction), mixed into waves with lanes that must pass through the rare branch unchanged
    pick = [0, 1, 2**32 - 1, 2**32 - 2, 0xFFFFFC2F, None, None]

    def limbmix():
        return sum((rng.getrandbits(32) if (c := rng.choice(pick)) is None else c) << (32 * i)
                   for i in range(8))
    for _ in range(20000):
        pairs.append((limbmix(), limbmix()))
    return pairs


def run(op, pairs):
    from bitcoinconsensus_amd import blib
    L = blib()
    n = len(pairs)
    a = pack([x for x, _ in pairs])
    b = pack([y for _, y in pairs])
    out = (ctypes.c_uint32 * (8 * n))()
    assert L.mi_fe_selftest(op, a, b, out, ctypes.c_size_t(n)) == 0
    return unpack(out, n)


@pytest.mark.gpu
@pytest.mark.parametrize("op,name,fn", [
    (0, "add", lambda a, b: a + b),
    (1, "sub", lambda a, b: a - b),
    (2, "mul", lambda a, b: a * b),
    (3, "sqr", lambda a, b: a * a),
    (4, "shl1", lambda a, b: 2 * a),
    (5, "shl2", lambda a, b: 4 * a),
    (6, "shl3", lambda a, b: 8 * a),
    (7, "neg", lambda a, b: -a),
])
def test_field_op_matches_integers(op, name, fn):
    pairs = operand_pairs()
    got = run(op, pairs)
    bad = [(i, a, b, g) for i, ((a, b), g) in enumerate(zip(pairs, got)) if g % P != fn(a, b) % P]
    assert not bad, f"{name}: {len(bad)} mismatches, first {bad[0]}"


@pytest.mark.gpu
def test_field_is_zero_and_normalize():
    vals = EDGES + [0, P, 2 * P - 2**256 + 2**256 - P] + [random.Random(3).getrandbits(256) for _ in range(2000)]
    pairs = [(v, 0) for v in vals]
    z = run(8, pairs)
    assert [g & 1 for g in z] == [1 if v % P == 0 else 0 for v in vals]
    nrm = run(9, pairs)
    assert nrm == [v % P for v in vals]


N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


@pytest.mark.gpu
def test_safegcd_inverses_match_integers():
    """The lanes' safegcd inverse (csrc/modinv_device.h: 30-bit branchless divstep batches, wave-
    uniform early exit) behind fe_inv (K_tfin) and sc_inv (K_inv): weak field operands (>= p
    included) and scalars < n, edge values and random lanes mixed in the same waves, against
    pow(a, -1, m); zero maps to zero as with the Fermat chains."""
    rng = random.Random(0x1417)
    fvals = EDGES + [rng.getrandbits(256) for _ in range(6000)]
    rng.shuffle(fvals)
    got = run(10, [(v, 0) for v in fvals])
    bad = [(v, g) for v, g in zip(fvals, got)
           if g != (pow(v % P, -1, P) if v % P else 0)]
    assert not bad, f"fe_inv: {len(bad)} mismatches, first {bad[0]}"
    svals = [0, 1, 2, N - 1, N - 2, (N + 1) // 2, 2**255 % N, 2**128] + \
        [rng.randrange(N) for _ in range(6000)]
    rng.shuffle(svals)
    got = run(11, [(v, 0) for v in svals])
    bad = [(v, g) for v, g in zip(svals, got) if g != (pow(v, -1, N) if v else 0)]
    assert not bad, f"sc_inv: {len(bad)} mismatches, first {bad[0]}"
