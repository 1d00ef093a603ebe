"""CPU: the proof behind the unguarded field products (round 6, tools/gen_fe_asm.py
mul_256x256_col_u / sqr_cross_col_u, secp256k1_device.h fe_mul / fe_sqr).

Each product column's first v_mad_u64_u32 adds its product to the previous column's carry words
and DROPS its carry out of bit 64.  The claim: with a[0] <= 2^32 - 9 and b[7] <= 2^32 - 9 (a[0] and
a[7] for a square's cross products) no first multiply-add can carry, so the unguarded columns are
exact; the kernels check those two limbs (a wave-wide ballot) and otherwise run the exact columns.
This emulates the generated column code instruction by instruction on Python integers:
* at the bound (and on random and all-ones-heavy operands within it) the unguarded product equals
  the integer product;
* just past the bound some operands make it wrong (so the check is needed, and the bound is tight
  enough to matter);
* the generated header really drops only the first carry of each column and has the column
  structure the proof assumes."""
import os
import random
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "rust-bitcoinconsensus_amd", "csrc", "fe_asm_gen.h")
M64 = (1 << 64) - 1
BOUND = (1 << 32) - 9


def mul_prods(k):
    return [(i, k - i) for i in range(max(0, k - 7), min(7, k) + 1)]


def cross_prods(k):
    return [(i, k - i) for i in range(max(0, k - 7), (k + 1) // 2)] if 1 <= k <= 13 else []


def columns_unguarded(a, b, prods, ncols):
    """The generated scheme: per column acc (64 bits) + nh (carry count); the first multiply-add's
    carry is dropped, every other one counted in nh.  Returns the column words and the exact flag
    (no first carry was dropped)."""
    acc, out, exact = 0, [], True
    for k in range(ncols):
        ps = prods(k)
        if not ps:
            out.append(None)
            continue
        nh = 0
        for n, (i, j) in enumerate(ps):
            s = a[i] * b[j] + acc
            if s > M64:
                if n == 0:
                    exact = False  # dropped
                else:
                    nh += 1
            acc = s & M64
        out.append(acc & 0xFFFFFFFF)
        acc = (acc >> 32) | (nh << 32)
    return out, acc, exact


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def value_mul(a, b):
    words, acc, _ = columns_unguarded(a, b, mul_prods, 15)
    t = words + [acc & 0xFFFFFFFF]  # t[15]: the last column's high word
    return sum(w << (32 * i) for i, w in enumerate(t))


def value_cross(a):
    words, acc, _ = columns_unguarded(a, a, cross_prods, 14)
    x = [0] + words[1:14] + [acc & 0xFFFFFFFF]
    return sum(w << (32 * i) for i, w in enumerate(x))


def cross_exact(a):
    return sum(a[i] * a[j] << (32 * (i + j)) for i in range(8) for j in range(i + 1, 8))


def operand(rng, lo_cap=None, hi_cap=None, ones=0.5):
    v = [0xFFFFFFFF if rng.random() < ones else rng.getrandbits(32) for _ in range(8)]
    if lo_cap is not None:
        v[0] = min(v[0], lo_cap)
    if hi_cap is not None:
        v[7] = min(v[7], hi_cap)
    return v


def test_unguarded_products_exact_within_the_bound():
    rng = random.Random(0xB0)
    for _ in range(20000):
        a = operand(rng, lo_cap=BOUND, ones=rng.choice((0.0, 0.5, 0.9, 1.0)))
        b = operand(rng, hi_cap=BOUND, ones=rng.choice((0.0, 0.5, 0.9, 1.0)))
        A = sum(w << (32 * i) for i, w in enumerate(a))
        Bv = sum(w << (32 * i) for i, w in enumerate(b))
        assert value_mul(a, b) == A * Bv
        s = operand(rng, lo_cap=BOUND, hi_cap=BOUND, ones=rng.choice((0.0, 0.9, 1.0)))
        assert value_cross(s) == cross_exact(s)
    # the worst case: every limb all-ones except the two checked ones at the bound
    a = [BOUND] + [0xFFFFFFFF] * 7
    b = [0xFFFFFFFF] * 7 + [BOUND]
    assert value_mul(a, b) == sum(w << (32 * i) for i, w in enumerate(a)) * \
        sum(w << (32 * i) for i, w in enumerate(b))
    s = [BOUND] + [0xFFFFFFFF] * 6 + [BOUND]
    assert value_cross(s) == cross_exact(s)


def test_unguarded_products_wrong_past_the_bound():
    """All-ones operands (a[0], b[7] past the bound) drop a carry: the check is not decorative."""
    a = b = [0xFFFFFFFF] * 8
    A = (1 << 256) - 1
    assert value_mul(a, b) != A * A
    assert value_cross(a) != cross_exact(a)


def test_generated_header_matches_the_proof():
    src = open(GEN).read()
    for fn, prods, ncols in (("mul_256x256_col_u", mul_prods, 15), ("sqr_cross_col_u", cross_prods, 14)):
        body = src[src.index(f"void {fn}("):]
        body = body[: body.index("\n}\n")]
        assert "%[f]" not in body and "ovf" not in body
        cols = re.findall(r'asm\("(.*?)" :', body)
        want = [k for k in range(ncols) if prods(k)]
        assert len(cols) == len(want), (fn, len(cols))
        for k, c in zip(want, cols):
            mads = re.findall(r"v_mad_u64_u32 %\[acc\], (vcc|%\[f\]), %\[(\w)(\d)\], %\[(\w)(\d)\]", c)
            pairs = [(int(x[2]), int(x[4])) for x in mads]
            assert pairs == prods(k), (fn, k, pairs)
            # every multiply-add after the first has its carry counted (an add-with-carry into nh)
            # unless the column is the last one
            addcs = c.count("v_addc_co_u32")
            assert addcs == (len(pairs) - 1 if k != want[-1] else 0), (fn, k, addcs)
