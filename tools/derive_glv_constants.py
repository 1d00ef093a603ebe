"""Derive the secp256k1 GLV-endomorphism constants used by csrc/secp256k1_device.h.

Independent derivation from the curve parameters (public math, Hankerson-Menezes-Vanstone
"Guide to ECC" alg. 3.74 with the rounded-multiplication estimate of Gouvea-Oliveira-Lopez):
  beta   : primitive cube root of unity mod p
  lambda : the cube root of unity mod n with lambda*(x, y) = (beta*x, y)
  (a1,b1),(a2,b2): short basis of {(a, b) : a + b*lambda == 0 mod n} from extended Euclid
  g1 = round(2^384 * b2 / n), g2 = round(2^384 * (-b1) / n)
Run: python3 tools/derive_glv_constants.py
"""
p = 2**256 - 2**32 - 977
n = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
Gx = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
Gy = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def add(P, Q):
    if P is None:
        return Q
    if Q is None:
        return P
    if P[0] == Q[0] and (P[1] + Q[1]) % p == 0:
        return None
    if P == Q:
        s = 3 * P[0] * P[0] * pow(2 * P[1], -1, p) % p
    else:
        s = (Q[1] - P[1]) * pow(Q[0] - P[0], -1, p) % p
    x = (s * s - P[0] - Q[0]) % p
    return (x, (s * (P[0] - x) - P[1]) % p)


def mul(k, P):
    R = None
    while k:
        if k & 1:
            R = add(R, P)
        P = add(P, P)
        k >>= 1
    return R


def cbrt1(m):
    for g in range(2, 100):
        r = pow(g, (m - 1) // 3, m)
        if r != 1:
            return r


def main():
    b0, l0 = cbrt1(p), cbrt1(n)
    beta = lam = None
    for l in (l0, l0 * l0 % n):
        L = mul(l, (Gx, Gy))
        for b in (b0, b0 * b0 % p):
            if L == (b * Gx % p, Gy):
                beta, lam = b, l
    assert beta is not None
    # extended Euclid on (n, lambda): remainders r_i with r_i == t_i * lambda (mod n)
    rs = [(n, 0), (lam, 1)]
    while rs[-1][0] * rs[-1][0] >= n:
        (r0, t0), (r1, t1) = rs[-2], rs[-1]
        q = r0 // r1
        rs.append((r0 - q * r1, t0 - q * t1))
    (rl, tl), (rl1, tl1) = rs[-2], rs[-1]
    q = rl // rl1
    rl2, tl2 = rl - q * rl1, tl - q * tl1
    a1, b1 = rl1, -tl1
    a2, b2 = min([(rl, -tl), (rl2, -tl2)], key=lambda v: v[0] ** 2 + v[1] ** 2)
    assert (a1 + b1 * lam) % n == 0 and (a2 + b2 * lam) % n == 0
    assert abs(a1 * b2 - b1 * a2) == n
    g1 = (2**384 * b2 + n // 2) // n
    g2 = (2**384 * (-b1) + n // 2) // n
    out = dict(beta=beta, lam=lam, a1=a1, b1=b1, a2=a2, b2=b2, g1=g1, g2=g2,
               minus_b1=(-b1) % n, minus_b2=(-b2) % n)
    for k, v in out.items():
        print(f"{k:9s} = {'-' if v < 0 else ''}0x{abs(v):064x}")
    return out


if __name__ == "__main__":
    main()
