"""Constants of csrc/fe29.h (radix-2^29 field): K48 (48 p with every limb raised above 2^29 + 2^27
by borrowing, the offset of fe9_sub) and p's canonical radix-2^29 digits.  Prints the C initialisers
and checks them."""
P = 2**256 - 2**32 - 977
M = 2**29


def balanced(k):
    r, d = k * P, []
    for _ in range(8):
        lo = r % M + M
        if lo < M + (1 << 27):
            lo += M
        d.append(lo)
        r = (r - lo) // M
    d.append(r)
    assert sum(v * M**i for i, v in enumerate(d)) == k * P
    return d


def digits(x):
    return [(x >> (29 * i)) & (M - 1) for i in range(9)]


if __name__ == "__main__":
    k48 = balanced(48)
    assert all(v >= M + 2 for v in k48) and all(v < 2**30 for v in k48)
    assert all(2 * v >= 2**30 + 2 for v in k48)
    print("K48 ", "{" + ", ".join(f"0x{v:08x}u" for v in k48) + "}")
    print("P29 ", "{" + ", ".join(f"0x{v:08x}u" for v in digits(P)) + "}")
    # fold identities used by fe9_reduce
    assert pow(2, 261, P) == 2**37 + 31264
    assert pow(2, 493, P) == (31264 * 2**232 + 65536 * 2**29 + 8003584) % P
